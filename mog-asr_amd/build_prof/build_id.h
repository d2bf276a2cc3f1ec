#define MOG_BUILD_ID "90b378e38f6fd0e0"
