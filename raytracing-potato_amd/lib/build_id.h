#define RP_BUILD_ID "d5e8b9da5e0643ae"
