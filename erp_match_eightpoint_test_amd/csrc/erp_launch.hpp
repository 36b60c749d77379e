// Kernel launch wrappers.  ERP_LAUNCH(kernel, grid, block, shmem, stream, args...) is
// hipLaunchKernelGGL; a build with -DERP_DEBUG_LAUNCH=1 also checks hipGetLastError() after
// every launch and returns the error from the enclosing launch_* function (hipError_t) at the
// launch that failed, naming it on stderr (release builds check once, at each launch_*'s end).
// ERP_LAUNCH_S is the same for entry points returning erp_status.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdio>

#ifndef ERP_DEBUG_LAUNCH
#define ERP_DEBUG_LAUNCH 0
#endif

#if ERP_DEBUG_LAUNCH
#define ERP_LAUNCH_IMPL(fail, kernel, ...)                                                   \
    do {                                                                                     \
        hipLaunchKernelGGL(kernel, __VA_ARGS__);                                             \
        const hipError_t erp_le_ = hipGetLastError();                                        \
        if (erp_le_ != hipSuccess) {                                                         \
            fprintf(stderr, "erp: launch of %s failed (%s:%d): %s\n", #kernel, __FILE__,      \
                    __LINE__, hipGetErrorString(erp_le_));                                   \
            return fail;                                                                     \
        }                                                                                    \
    } while (0)
#define ERP_LAUNCH(kernel, ...) ERP_LAUNCH_IMPL(erp_le_, kernel, __VA_ARGS__)
#define ERP_LAUNCH_S(kernel, ...) ERP_LAUNCH_IMPL(ERP_HIP_ERROR, kernel, __VA_ARGS__)
#else
#define ERP_LAUNCH(kernel, ...) hipLaunchKernelGGL(kernel, __VA_ARGS__)
#define ERP_LAUNCH_S(kernel, ...) hipLaunchKernelGGL(kernel, __VA_ARGS__)
#endif
