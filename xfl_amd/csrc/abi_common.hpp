// Shared by the two translation units of libxhe.so (xhe.hip: device code and
// the kernel entry points; wire_abi.cpp: host-only entry points): the
// thread-local error message behind xhe_last_error().
#pragma once
#include <string>

// Records msg as this thread's last error and returns code.
int xhe_fail(int code, const std::string& msg);
