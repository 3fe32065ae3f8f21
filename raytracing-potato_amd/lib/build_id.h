#define RP_BUILD_ID "ec12f559726a6fda"
