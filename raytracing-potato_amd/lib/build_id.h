#define RP_BUILD_ID "e9be37cfc887f1e8"
