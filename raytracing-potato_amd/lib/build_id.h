#define RP_BUILD_ID "14a0538f7cbb422c"
