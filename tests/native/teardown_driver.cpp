// Teardown check of libmsm's host thread pools, built with a sanitizer (make -C webgpu-msm_amd
// sanitize; tests/test_teardown.py runs it, no GPU needed).  Starts every pool the library keeps
// (packing threads, lone-MSM tail helpers, pipelined-tail threads) at the sizes for 1, 2 and 8
// devices, then exits: mode 0 after msm_shutdown (what the Python binding's atexit handler and the
// Node addon's cleanup hook call), mode 1 without it (parked threads at process exit).
#include <cstdio>
#include <cstdlib>
#include <initializer_list>

#include "../../include/msm.h"

extern "C" int msm_test_pools(int ndev, int run, int* out);

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  int out[5];
  for (int nd : {1, 2, 8, 1}) {
    const int rc = msm_test_pools(nd, 1, out);
    if (rc != 0) {
      fprintf(stderr, "msm_test_pools(%d) = %d\n", nd, rc);
      return 2;
    }
    printf("devices %d: budget %d pack %d tail %d horner %d total %d\n", nd, out[0], out[1], out[2], out[3], out[4]);
  }
  if (mode == 0) msm_shutdown();
  return 0;
}
