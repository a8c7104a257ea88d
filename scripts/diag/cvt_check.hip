// Diagnostic: does the packed fp32 -> fp16 conversion the compiler emits for a half4 built from
// four casts round like the scalar one? Writes both, per input, for a sweep of values near
// fp16 rounding midpoints.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
__global__ void cvt(const float* x, half4* packed, _Float16* lo, _Float16* scalar, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (4 * i + 3 >= n) return;
  half4 a;
  for (int r = 0; r < 4; ++r) a[r] = (_Float16)x[4 * i + r];
  packed[i] = a;
  for (int r = 0; r < 4; ++r) lo[4 * i + r] = (_Float16)(x[4 * i + r] - (float)a[r]);
  volatile float v = x[4 * i];
  scalar[4 * i] = (_Float16)v;
}
int main() {
  const int n = 1 << 20;
  float* hx = (float*)malloc(n * 4);
  srand(1);
  for (int i = 0; i < n; ++i) hx[i] = ((float)rand() / RAND_MAX * 2.f - 1.f);
  float *dx; half4* dp; _Float16 *dl, *ds;
  hipMalloc(&dx, n * 4); hipMalloc(&dp, n * 2); hipMalloc(&dl, n * 2); hipMalloc(&ds, n * 2);
  hipMemcpy(dx, hx, n * 4, hipMemcpyHostToDevice);
  hipMemset(ds, 0, n * 2);
  cvt<<<n / 4 / 256, 256>>>(dx, dp, dl, ds, n);
  _Float16* hp = (_Float16*)malloc(n * 2); _Float16* hl = (_Float16*)malloc(n * 2);
  _Float16* hs = (_Float16*)malloc(n * 2);
  hipMemcpy(hp, dp, n * 2, hipMemcpyDeviceToHost); hipMemcpy(hl, dl, n * 2, hipMemcpyDeviceToHost);
  hipMemcpy(hs, ds, n * 2, hipMemcpyDeviceToHost);
  int bad_hi = 0, bad_lo = 0, bad_sc = 0;
  for (int i = 0; i < n; ++i) {
    const float x = hx[i];
    const _Float16 rne = (_Float16)x;            // host conversion: RNE
    if ((float)hp[i] != (float)rne) { if (bad_hi < 5) printf("packed %d: x %.9g got %.9g rne %.9g\n", i, x, (float)hp[i], (float)rne); ++bad_hi; }
    const float want_lo = (float)(_Float16)(x - (float)hp[i]);
    if ((float)hl[i] != want_lo) { if (bad_lo < 5) printf("lo %d: x %.9g hi %.9g lo %.9g want %.9g\n", i, x, (float)hp[i], (float)hl[i], want_lo); ++bad_lo; }
    if (i % 4 == 0 && (float)hs[i] != (float)rne) ++bad_sc;
  }
  printf("n %d  packed!=rne %d  lo inconsistent with stored hi %d  scalar!=rne %d\n", n, bad_hi, bad_lo, bad_sc);
  return 0;
}
