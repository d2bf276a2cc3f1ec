#define MOG_BUILD_ID "339fa036a2ccd2e6"
