#define MOG_BUILD_ID "8c6f1e38a6b5d2e4"
