// Every kernel unit linked into libmrbo.so must have been compiled against the host API's KParams
// layout (a unit compiled from an older mrbo_device.h reads every launch parameter at a shifted
// offset).  Built and run by tests/test_host.py on the CPU: kset_d*() only takes kernel addresses.
#include "mrbo_dispatch.h"
#include <cstdio>
using namespace mrbo;
int main() {
  int bad = 0, n = 0;
#define CHK(FN, DD) { KernelSet ks; for (int r : {1, 2, 4, 8}) if (FN(r, ks)) { ++n; if (ks.kparams_bytes != sizeof(KParams)) { ++bad; printf("unit %s rpl %d: %zu vs %zu\n", #FN, r, ks.kparams_bytes, sizeof(KParams)); } } }
#define K6(DD) CHK(kset_d##DD, DD)
#define K4(DD) CHK(kset_d##DD##_f4, DD)
  K6(1) K6(2) K6(3) K6(4) K6(5) K6(6) K6(7) K6(8) K6(9) K6(10) K6(12) K6(16)
  K4(1) K4(2) K4(3) K4(4) K4(6) K4(8)
  printf("checked %d kernel sets, %d mismatched, sizeof(KParams) = %zu\n", n, bad, sizeof(KParams));
  return bad != 0;
}
