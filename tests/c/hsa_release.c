/* The ROCr release parser and query of csrc/runtime.c, compiled in (the parser
 * is not exported).  Prints "parser ok" and the queried release / bound. */
#define _GNU_SOURCE
#include <stdarg.h>
#include <stdio.h>

int inccl_set_error(int rc, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
    return rc;
}

#include "../../container_inc_amd/csrc/runtime.c"

int main(void)
{
    static const struct { const char *s; unsigned want; } cases[] = {
        {"\"1.18.0-rocm-rel-7.2-43-fc0010cf6a\"", 702},   /* /opt/rocm on the MI355X box */
        {"\"1.18.0-rocm-rel-7.0-56-b59f6da2\"", 700},     /* PyTorch's bundled ROCr */
        {"1.20.0-rocm-rel-10.1-1-x", 1001},
        {"1.18.0-rocm-rel-7", 0},
        {"1.18.0", 0},
        {"", 0},
        {NULL, 0},
    };
    for (unsigned i = 0; i < sizeof(cases) / sizeof(cases[0]); ++i)
        if (inccl_hsa_release_of(cases[i].s) != cases[i].want) {
            printf("parser FAILED on %s: %u\n", cases[i].s ? cases[i].s : "(null)", inccl_hsa_release_of(cases[i].s));
            return 1;
        }
    printf("parser ok\nrelease %u build %s bound %zu\n", inccl_hsa_runtime_release(), inccl_hsa_runtime_build(),
           inccl_ipc_local_max_bytes());
    return 0;
}
