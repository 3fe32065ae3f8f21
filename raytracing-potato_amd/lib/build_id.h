#define RP_BUILD_ID "9da3ce01dfd95a72"
