#define RP_BUILD_ID "ff7fd58c2e5269af"
