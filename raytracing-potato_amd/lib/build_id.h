#define RP_BUILD_ID "13c06ba3cbadb017"
