/* runtime.c -- which HSA runtime this process runs on, and what it allows.
 *
 * Importing a peer's IPC allocation larger than 2 GiB (hipIpcOpenMemHandle of
 * a dmabuf export) never returns under the HSA runtime (ROCr) that PyTorch
 * bundles (ROCm 7.0.2), whatever the HIP runtime above it; under /opt/rocm's
 * ROCm 7.2 ROCr it works.  Established by mixing the layers in a two-process C
 * probe: HIP 7.0 over HSA 7.2 imports 2.6 GB, HIP 7.2 over HSA 7.0 hangs
 * (DESIGN.md "2 GiB per IPC export", profiles/r03/ipc_probe/).
 *
 * So the largest single IPC export depends on the ROCm release of the HSA
 * runtime the process has mapped.  The runtime itself is asked: the mapped
 * libhsa-runtime64 is found (dl_iterate_phdr), its own hsa_system_get_info
 * answers HSA_AMD_SYSTEM_INFO_BUILD_VERSION, a string such as
 * "1.18.0-rocm-rel-7.2-43-fc0010cf6a" (/opt/rocm) or "1.18.0-rocm-rel-7.0-56-
 * b59f6da2" (torch's; profiles/r04/rehearse_n8/hsa_build_probe.txt).  Release
 * 7.2 or later gets no bound; an older one, a build string without a release
 * tag, or a runtime that cannot be asked (no GPU) keeps every export below
 * 2 GiB.  $INCCL_IPC_MAX_BYTES overrides (rounded down to whole MiB, at least
 * 1 MiB).  The answer is computed once per process (pthread_once).  A group
 * agrees on the smallest bound over its ranks at creation, so every rank
 * refuses (or not) alike.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <limits.h>
#include <link.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <rccl/rccl.h>

#include "inccl_internal.h"

#define HSA_AMD_SYSTEM_INFO_BUILD_VERSION_ATTR 0x200   /* hsa.h: a const char* */

static int find_hsa(struct dl_phdr_info *info, size_t size, void *data)
{
    (void)size;
    const char *n = info->dlpi_name;
    if (n && strstr(n, "libhsa-runtime64")) {
        snprintf((char *)data, PATH_MAX, "%s", n);
        return 1;
    }
    return 0;
}

/* "...-rocm-rel-<major>.<minor>-..." -> major * 100 + minor; 0 without the tag */
unsigned inccl_hsa_release_of(const char *build)
{
    const char *v = build ? strstr(build, "rocm-rel-") : NULL;
    unsigned major = 0, minor = 0;
    if (!v || sscanf(v, "rocm-rel-%u.%u", &major, &minor) != 2 || minor > 99) return 0;
    return major * 100 + minor;
}

static unsigned g_release;
static char g_build[128];
static pthread_once_t g_release_once = PTHREAD_ONCE_INIT;

typedef int (*hsa_status_fn)(void);
typedef int (*hsa_info_fn)(int, void *);

static void query_release(void)
{
    char path[PATH_MAX] = "";
    if (hipInit(0) != hipSuccess) return;   /* no GPU: nothing to ask, the bound stays */
    dl_iterate_phdr(find_hsa, path);
    if (!path[0]) return;
    void *h = dlopen(path, RTLD_NOW | RTLD_NOLOAD);   /* the copy already mapped, not another */
    if (!h) return;
    hsa_status_fn init = (hsa_status_fn)dlsym(h, "hsa_init");
    hsa_status_fn shut = (hsa_status_fn)dlsym(h, "hsa_shut_down");
    hsa_info_fn info = (hsa_info_fn)dlsym(h, "hsa_system_get_info");
    if (init && shut && info && init() == 0) {   /* reference-counted: HIP holds its own */
        const char *b = NULL;
        if (info(HSA_AMD_SYSTEM_INFO_BUILD_VERSION_ATTR, &b) == 0 && b) {
            /* the string comes quoted ("\"1.18.0-rocm-rel-7.0-...\""): kept without the quotes */
            const size_t n = strlen(b);
            const int q = n >= 2 && b[0] == '"' && b[n - 1] == '"';
            snprintf(g_build, sizeof(g_build), "%.*s", (int)(q ? n - 2 : n), q ? b + 1 : b);
            g_release = inccl_hsa_release_of(b);
        }
        shut();
    }
    dlclose(h);
}

unsigned inccl_hsa_runtime_release(void)
{
    pthread_once(&g_release_once, query_release);
    return g_release;
}

const char *inccl_hsa_runtime_build(void)
{
    pthread_once(&g_release_once, query_release);
    return g_build;
}

size_t inccl_ipc_local_max_bytes(void)
{
    const char *e = getenv("INCCL_IPC_MAX_BYTES");
    if (e && *e) {
        const unsigned long long v = strtoull(e, NULL, 0) >> 20 << 20;   /* whole MiB, as the group agrees */
        if (v >= (1ull << 20)) return (size_t)v;
        fprintf(stderr, "inccl: INCCL_IPC_MAX_BYTES=%s is below 1 MiB; ignored\n", e);
    }
    return inccl_hsa_runtime_release() >= 702u ? INCCL_IPC_MAX_BYTES_UNBOUNDED : INCCL_IPC_MAX_BYTES_DEFAULT;
}

size_t inccl_ipc_max_bytes(void) { return inccl_ipc_local_max_bytes(); }

size_t inccl_group_ipc_max_bytes(const struct inccl_group *g) { return g ? g->ipc_max_bytes : 0; }

int inccl_rccl_version(int *compiled, int *loaded)
{
    if (compiled) *compiled = NCCL_VERSION_CODE;
    int v = 0;
    const ncclResult_t r = ncclGetVersion(&v);
    if (loaded) *loaded = r == ncclSuccess ? v : 0;
    return r == ncclSuccess ? 0 : inccl_set_error(INCCL_ERR_NCCL, "ncclGetVersion: %s", ncclGetErrorString(r));
}
