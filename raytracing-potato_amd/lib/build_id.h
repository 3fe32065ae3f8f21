#define RP_BUILD_ID "5537149adc242ddd"
