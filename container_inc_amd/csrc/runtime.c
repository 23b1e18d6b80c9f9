/* runtime.c -- which HSA runtime this process runs on, and what it allows.
 *
 * Importing a peer's IPC allocation larger than 2 GiB (hipIpcOpenMemHandle of
 * a dmabuf export) never returns under the HSA runtime (ROCr) that PyTorch
 * bundles (ROCm 7.0.2), whatever the HIP runtime above it; under /opt/rocm's
 * ROCm 7.2 ROCr it works.  Established by mixing the layers in a two-process C
 * probe: HIP 7.0 over HSA 7.2 imports 2.6 GB, HIP 7.2 over HSA 7.0 hangs
 * (DESIGN.md "2 GiB per IPC export", profiles/r03/ipc_probe/).
 *
 * So the largest single IPC export depends on the HSA runtime the process has
 * mapped: a ROCr whose file carries a ROCm build >= 7.2 (libhsa-runtime64.so.1.
 * <minor>.<build>, build >= 70200) gets no bound; any other (torch's file is
 * unversioned) keeps every export below 2 GiB.  $INCCL_IPC_MAX_BYTES overrides.
 * A group agrees on the smallest bound over its ranks at creation, so every
 * rank refuses (or not) alike.
 */
#define _GNU_SOURCE
#include <limits.h>
#include <link.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "inccl_internal.h"

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

/* Real path of the mapped HSA runtime, or "" (none mapped). */
const char *inccl_hsa_runtime_path(void)
{
    static char real[PATH_MAX];
    char path[PATH_MAX] = "";
    dl_iterate_phdr(find_hsa, path);
    if (!path[0]) return "";
    if (!realpath(path, real)) snprintf(real, sizeof(real), "%s", path);
    return real;
}

/* The ROCm build number in a ROCr file name (libhsa-runtime64.so.1.18.70200 ->
 * 70200), or 0 when the name carries none. */
unsigned inccl_hsa_build_of(const char *path)
{
    const char *b = strrchr(path, '/');
    b = b ? b + 1 : path;
    const char *v = strstr(b, "libhsa-runtime64.so.");
    if (!v) return 0;
    unsigned major = 0, minor = 0, build = 0;
    if (sscanf(v, "libhsa-runtime64.so.%u.%u.%u", &major, &minor, &build) != 3) return 0;
    return build;
}

size_t inccl_ipc_local_max_bytes(void)
{
    const char *e = getenv("INCCL_IPC_MAX_BYTES");
    const unsigned long long v = e ? strtoull(e, NULL, 0) : 0;
    if (v) return (size_t)v;
    return inccl_hsa_build_of(inccl_hsa_runtime_path()) >= 70200u ? INCCL_IPC_MAX_BYTES_UNBOUNDED
                                                                   : INCCL_IPC_MAX_BYTES_DEFAULT;
}

size_t inccl_ipc_max_bytes(void) { return inccl_ipc_local_max_bytes(); }

size_t inccl_group_ipc_max_bytes(const struct inccl_group *g) { return g ? g->ipc_max_bytes : 0; }
