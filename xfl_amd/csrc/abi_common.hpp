// Shared by the two translation units of libxhe.so (xhe.hip: device code and
// the kernel entry points; wire_abi.cpp: host-only entry points): the
// thread-local error message behind xhe_last_error().
#pragma once
#include <stdint.h>

#include <string>

// Records msg as this thread's last error and returns code.
int xhe_fail(int code, const std::string& msg);

// memcpy of n bytes split over the host's codec threads (at most 16, the
// GPU box's CPU share per GPU) when n is large; the destination pages are
// first touched by those threads, so fresh pageable memory faults in
// parallel. Defined in wire_abi.cpp.
void xhe_host_copy(void* dst, const void* src, int64_t n);
