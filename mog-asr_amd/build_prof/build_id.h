#define MOG_BUILD_ID "ca2c22374b1b1d55"
