#define RP_BUILD_ID "96aa69cf214ccf75"
