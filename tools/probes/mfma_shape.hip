// MFMA shape probe (VERDICT r4 "next round" item 2): does v_mfma_f32_32x32x16_bf16 feed a
// GEMM main loop better than the v_mfma_f32_16x16x32_bf16 every bf16 kernel here uses?
//
// Each wave owns the 8-phase GEMM kernel's per-wave piece, a 32 x 64 output tile, and per
// iteration consumes one BK = 64 slice of LDS-resident, k-contiguous operand images
// (A [32][64], B [64][64] bf16, rows padded to 144 B: conflict-free 16-lane ds_read_b128):
//   shape 0: 2 x 4 tiles of 16x16 x 2 k-halves = 16 MFMAs of 16x16x32, 12 ds_read_b128
//   shape 1: 1 x 2 tiles of 32x32 x 4 k-steps  =  8 MFMAs of 32x32x16, 12 ds_read_b128
// -- the same operand bytes per FLOP (a wave reads its tile's A rows and B columns once per k
// whatever the MFMA shape), so what differs is the instruction stream and the clock the chip
// holds.  Random operands (MI355X_MICROARCH.md: zeros run a higher clock).  Full chip: 256
// blocks x W waves (W / 4 per SIMD), each wave on its own LDS image.
//
//   hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_shape.hip -o build/mfma_shape
//   build/mfma_shape            -> one JSON line per (shape, waves per SIMD)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int PITCH = 72;  // bf16 per LDS row: 64 + 8 (144 B)
constexpr int IMG = (32 + 64) * PITCH;  // one wave's A + B image (bf16 elements)

template <int SHAPE, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void mfma_loop(const __bf16* __restrict__ src,
                                                        float* __restrict__ out, int iters) {
  __shared__ __bf16 lds[WAVES * IMG];
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  for (int i = t; i < WAVES * IMG; i += 64 * WAVES) lds[i] = src[(blockIdx.x * 7919 + i) & 0xFFFFF];
  __syncthreads();
  const __bf16* A = lds + wave * IMG;
  const __bf16* Bm = A + 32 * PITCH;
  if constexpr (SHAPE == 0) {
    f32x4 acc[2][4] = {};
    const int r = lane & 15, kq = (lane >> 4) * 8;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        bfx8 a[2], b[4];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = *(const bfx8*)(A + (i * 16 + r) * PITCH + kh * 32 + kq);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = *(const bfx8*)(Bm + (j * 16 + r) * PITCH + kh * 32 + kq);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    out[blockIdx.x * 64 * WAVES + t] = s;
  } else {
    f32x16 acc[2] = {};
    const int r = lane & 31, kq = (lane >> 5) * 8;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bfx8 a = *(const bfx8*)(A + r * PITCH + ks * 16 + kq);
        bfx8 b[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] = *(const bfx8*)(Bm + (j * 32 + r) * PITCH + ks * 16 + kq);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[j], acc[j], 0, 0, 0);
      }
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) s += acc[j][e];
    out[blockIdx.x * 64 * WAVES + t] = s;
  }
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

template <int SHAPE, int WAVES>
void run(const __bf16* src, float* out, int iters) {
  const int blocks = 256;
  auto launch = [&] { hipLaunchKernelGGL((mfma_loop<SHAPE, WAVES>), dim3(blocks), dim3(64 * WAVES), 0, 0, src, out, iters); };
  for (int i = 0; i < 200; ++i) launch();  // >= 2 s of back-to-back work before timing
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 50;
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double flop = 2.0 * 32 * 64 * 64 * (double)iters * WAVES * blocks * reps;
  printf("{\"mfma\": \"%s\", \"waves_per_simd\": %d, \"iters\": %d, \"us_per_launch\": %.1f, "
         "\"tflops\": %.1f}\n",
         SHAPE == 0 ? "16x16x32_bf16" : "32x32x16_bf16", WAVES / 4, iters, ms * 1e3 / reps,
         flop / (ms * 1e-3) / 1e12);
  fflush(stdout);
}

int main() {
  const size_t n = 1 << 20;
  std::vector<unsigned short> h(n);
  unsigned s = 12345;
  for (auto& v : h) {  // random bf16 in about [-2, 2]
    s = s * 1664525u + 1013904223u;
    v = (unsigned short)(0x3F00 + ((s >> 16) & 0xFF) - 0x40) | ((s & 0x8000) ? 0x8000 : 0);
  }
  __bf16* src;
  float* out;
  CK(hipMalloc(&src, n * 2));
  CK(hipMalloc(&out, 256 * 512 * 4));
  CK(hipMemcpy(src, h.data(), n * 2, hipMemcpyHostToDevice));
  const int iters = 4000;
  for (int rep = 0; rep < 2; ++rep) {  // interleaved, twice
    run<0, 4>(src, out, iters);
    run<1, 4>(src, out, iters);
    run<0, 8>(src, out, iters);
    run<1, 8>(src, out, iters);
  }
  CK(hipFree(src));
  CK(hipFree(out));
  return 0;
}
