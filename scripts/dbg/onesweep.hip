// Diagnostic: rocPRIM's Onesweep radix sort (merge-sort limit 0) on the contribution-list
// shape of C3 at B = 8192 (855k int32 (key, slot) pairs, keys < 2^17), with the workspace
// queried by the same config.  Plain stream first, then captured into a hipGraph and
// replayed; each result checked against a stable host sort.  Prints one line per mode.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

using Cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 855000;
  const int T = 82174, bits = 17;
  std::mt19937 rng(1);
  std::vector<int> keys(n), vals(n);
  for (int i = 0; i < n; ++i) { keys[i] = (int)(rng() % (T + 1)); vals[i] = i; }
  std::vector<int> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return keys[a] < keys[b]; });
  int *dk, *dv, *sk, *sv;
  CK(hipMalloc(&dk, n * 4)); CK(hipMalloc(&dv, n * 4)); CK(hipMalloc(&sk, n * 4)); CK(hipMalloc(&sv, n * 4));
  CK(hipMemcpy(dk, keys.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dv, vals.data(), n * 4, hipMemcpyHostToDevice));
  size_t bytes = 0;
  CK(rocprim::radix_sort_pairs<Cfg>(nullptr, bytes, dk, sk, dv, sv, (size_t)n, 0, bits, (hipStream_t)0));
  void* tmp;
  CK(hipMalloc(&tmp, bytes));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  auto check = [&](const char* what) {
    std::vector<int> ok(n), ov(n);
    if (hipMemcpy(ok.data(), sk, n * 4, hipMemcpyDeviceToHost) != hipSuccess) { printf("%s: copy failed\n", what); return; }
    (void)hipMemcpy(ov.data(), sv, n * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; ++i) bad += (ov[i] != idx[i]) || (ok[i] != keys[idx[i]]);
    printf("%s: n=%d tmp=%zu bytes, mismatches %d\n", what, n, bytes, bad);
    (void)hipMemset(sk, 0, n * 4); (void)hipMemset(sv, 0, n * 4);
  };
  CK(rocprim::radix_sort_pairs<Cfg>(tmp, bytes, dk, sk, dv, sv, (size_t)n, 0, bits, s));
  CK(hipStreamSynchronize(s));
  check("stream");
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  CK(rocprim::radix_sort_pairs<Cfg>(tmp, bytes, dk, sk, dv, sv, (size_t)n, 0, bits, s));
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int r = 0; r < 3; ++r) {
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    check("graph replay");
  }
  return 0;
}
