// Shared HIP host-side helpers for the engine's kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <vector>

// Return the hipError_t (as int) from the enclosing int-returning function on failure.
#define BCC_HIP_TRY(expr)                                                                   \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) {                                                             \
            fprintf(stderr, "[bcc] HIP error %d (%s) at %s:%d: %s\n", (int)_e,              \
                    hipGetErrorString(_e), __FILE__, __LINE__, #expr);                      \
            return (int)_e;                                                                 \
        }                                                                                   \
    } while (0)
