#define RP_BUILD_ID "edeb3da151eb1761"
