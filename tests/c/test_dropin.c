/* A plain C consumer of include/kungfu_amd.h, linked with -lkungfu_amd:
 * the reference's own unit checks (tests/cpp/unit/test_kungfu.cpp:3-20,
 * test_operations.cpp:3-26 at np = 1) restated against the drop-in, plus the
 * device bucket API. Needs a GPU for the transform calls; exit code 0 = pass.
 *   gcc -I include tests/c/test_dropin.c -L kungfu_amd -lkungfu_amd \
 *       -Wl,-rpath,$PWD/kungfu_amd -o /tmp/test_dropin && /tmp/test_dropin  */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "kungfu_amd.h"

#define CHECK(c)                                                               \
    do {                                                                       \
        if (!(c)) {                                                            \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);       \
            return 1;                                                          \
        }                                                                      \
    } while (0)

int main(void)
{
    /* test_type_size */
    CHECK(kungfu_type_size(KungFu_INT32) == 4);
    CHECK(kungfu_type_size(KungFu_FLOAT16) == 2);
    CHECK(kungfu_type_size(KungFu_FLOAT) == 4);
    CHECK(kungfu_type_size(KungFu_DOUBLE) == 8);
    if (kf_device_count() < 1) {
        printf("no device: skipping transform checks\n");
        return 77;
    }
    /* test_transform: 1 + 2 = 3 in place into x */
    float x = 1, y = 2;
    std_transform_2(&x, &y, &x, 1, KungFu_FLOAT, KungFu_SUM);
    CHECK(x == 3.0f);
    /* int32 MIN/MAX/PROD, larger n */
    enum { N = 100000 };
    int *a = malloc(N * sizeof(int)), *b = malloc(N * sizeof(int)), *c = malloc(N * sizeof(int));
    for (int i = 0; i < N; ++i) {
        a[i] = i - 500;
        b[i] = 3 * (i % 77) - 100;
    }
    std_transform_2(a, b, c, N, KungFu_INT32, KungFu_MIN);
    for (int i = 0; i < N; ++i) CHECK(c[i] == (b[i] < a[i] ? b[i] : a[i]));
    std_transform_2(a, b, c, N, KungFu_INT32, KungFu_PROD);
    for (int i = 0; i < N; ++i) CHECK(c[i] == (int)((unsigned)a[i] * (unsigned)b[i]));
    /* np = 1 session: all-reduce is a copy (test_operations.cpp: y[i] == i+1) */
    kf_session_t *s = kf_session_create(0, 1, "/tmp", 0, 0);
    CHECK(s != NULL);
    for (int i = 0; i < 100; ++i) a[i] = i + 1;
    memset(c, 0, 100 * sizeof(int));
    CHECK(kf_session_all_reduce(s, a, c, 100, KungFu_INT32, KungFu_SUM, "test", NULL) == KF_OK);
    for (int i = 0; i < 100; ++i) CHECK(c[i] == i + 1);
    kf_session_destroy(s);
    free(a);
    free(b);
    free(c);
    CHECK(kf_shutdown() == KF_OK); /* HIP resources back while the runtime is up */
    printf("ok\n");
    return 0;
}
