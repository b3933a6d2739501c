extern "C"
int hetu_runtime_version() { return 1; }
