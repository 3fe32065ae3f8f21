#define RP_BUILD_ID "ae375ea43caf0676"
