#define RP_BUILD_ID "67fcd69d1b2a6ff4"
