#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));
struct C { float a[2][8]; };
__global__ void kpk(const C* __restrict__ c, const float* __restrict__ x, float* out) {
  int i = threadIdx.x + blockIdx.x * 64;
  v2f v = {x[i], x[i] * 2.0f};
  v2f acc = {0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    v2f ck = {c->a[0][k], c->a[1][k]};
    acc = v * ck + acc;       // v_pk_fma_f32 with SGPR pair?
    v = v * v2f{0.5f, 0.25f} + ck;
  }
  out[2 * i] = acc.x;
  out[2 * i + 1] = acc.y;
}
__global__ void ksc(const C* __restrict__ c, const float* __restrict__ x, float* out) {
  int i = threadIdx.x + blockIdx.x * 64;
  float v0 = x[i], v1 = x[i] * 2.0f, a0 = 0, a1 = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a0 = fmaf(v0, c->a[0][k], a0); a1 = fmaf(v1, c->a[1][k], a1);
    v0 = fmaf(v0, 0.5f, c->a[0][k]); v1 = fmaf(v1, 0.25f, c->a[1][k]);
  }
  out[2 * i] = a0; out[2 * i + 1] = a1;
}
int main() {
  C h; for (int a = 0; a < 2; ++a) for (int k = 0; k < 8; ++k) h.a[a][k] = (k % 3 == 0) ? 0.f : 0.1f * (k + 1) + a;
  C* dc; float *dx, *o1, *o2; hipMalloc(&dc, sizeof(C)); hipMalloc(&dx, 256 * 4); hipMalloc(&o1, 512 * 4); hipMalloc(&o2, 512 * 4);
  hipMemcpy(dc, &h, sizeof(C), hipMemcpyHostToDevice);
  float hx[256]; for (int i = 0; i < 256; ++i) hx[i] = 0.01f * i; hipMemcpy(dx, hx, 1024, hipMemcpyHostToDevice);
  kpk<<<4, 64>>>(dc, dx, o1); ksc<<<4, 64>>>(dc, dx, o2);
  float r1[512], r2[512]; hipMemcpy(r1, o1, 2048, hipMemcpyDeviceToHost); hipMemcpy(r2, o2, 2048, hipMemcpyDeviceToHost);
  double md = 0; for (int i = 0; i < 512; ++i) md = fmax(md, fabs(r1[i] - r2[i]));
  printf("max diff packed vs scalar %g  (r1[1]=%g r2[1]=%g)\n", md, r1[1], r2[1]);
}
