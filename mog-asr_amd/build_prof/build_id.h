#define MOG_BUILD_ID "04e17c3b3e5eaa98"
