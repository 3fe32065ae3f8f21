#define RP_BUILD_ID "debd61d00120727f"
