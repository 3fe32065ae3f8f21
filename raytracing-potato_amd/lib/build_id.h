#define RP_BUILD_ID "ab01c2b8503132aa"
