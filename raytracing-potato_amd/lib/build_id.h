#define RP_BUILD_ID "acbbfb2c68f12470"
