#define RP_BUILD_ID "2cbb61fcbc0f507c"
