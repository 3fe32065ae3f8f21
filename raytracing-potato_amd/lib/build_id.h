#define RP_BUILD_ID "86181f92ded443df"
