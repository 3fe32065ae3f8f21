#define RP_BUILD_ID "bf2f1ca6e02a35e1"
