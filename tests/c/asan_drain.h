// asan_drain.h — for the C/C++ test hosts under AddressSanitizer
// (tools/sanitize_gpu_hosts.sh). No effect in other builds.
//
// ASan keeps every freed chunk in a quarantine (256 MiB on x86-64) and frees
// the oldest when it overflows — the chunks of its DEVICE allocator too,
// i.e. every hipFree of the run. At exit, libamdhip64's own destructors
// (__cxa_finalize) unload the HSA runtime and then free host objects; if such
// a free pushes a device chunk out of the quarantine after the unload, ASan
// stops on CHECK "!dev_runtime_unloaded_" (sanitizer_allocator_device.h:125;
// round 4's raw log, profiles/r04/asan_check_r04c.log: no frame of this
// project on that stack). Called after the host's last device free,
// kf_asan_drain_quarantine cycles the quarantine with host chunks, so every
// device chunk leaves it while the runtime is still loaded.
#pragma once
#include <stdlib.h>
#include <string.h>

#if defined(__has_feature)
#if __has_feature(address_sanitizer)
#define KF_UNDER_ASAN 1
#endif
#endif
#if defined(__SANITIZE_ADDRESS__)
#define KF_UNDER_ASAN 1
#endif

static inline void kf_asan_drain_quarantine(void)
{
#ifdef KF_UNDER_ASAN
    for (int i = 0; i < 640; ++i) { /* 640 MiB: past any quarantine size in use */
        char *p = (char *)malloc(1 << 20);
        if (!p) break;
        memset(p, 0, 64);
        free(p);
    }
#endif
}
