#define RP_BUILD_ID "f3d668241d2aac0a"
