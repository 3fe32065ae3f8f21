#define RP_BUILD_ID "8ea710addda81833"
