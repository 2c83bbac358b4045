// Probe of v_mfma_scale_f32_16x16x128_f8f6f4 operand layout (one wave).
// Writes per case: the raw lane operands (a, b: 64 lanes x 32 bytes; scales:
// 64 lanes x 1 byte) and the result (64 lanes x 4 floats) to a binary file,
// analysed on the host (tools/mx_probe_analyze.py).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const i32x8* a, const i32x8* b, const int* sa, const int* sb, f32x4* d) {
  const int l = threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 0, 0, 0, sa[l], 0, sb[l]);
  d[l] = acc;
}

static unsigned char enc(int v) {  // small integer -> e4m3 byte (|v| <= 7)
  if (v == 0) return 0;
  int s = v < 0 ? 0x80 : 0;
  int a = v < 0 ? -v : v;
  int e = 0;
  while ((a >> (e + 1)) != 0) ++e;
  int m = ((a << 3) >> e) & 7;
  return (unsigned char)(s | ((e + 7) << 3) | m);
}

int main(int argc, char** argv) {
  const char* out = argc > 1 ? argv[1] : "mx_probe.bin";
  FILE* f = fopen(out, "wb");
  srand(1);
  i32x8 *da, *db;
  int *dsa, *dsb;
  f32x4* dd;
  hipMalloc(&da, 64 * 32);
  hipMalloc(&db, 64 * 32);
  hipMalloc(&dsa, 64 * 4);
  hipMalloc(&dsb, 64 * 4);
  hipMalloc(&dd, 64 * 16);
  for (int c = 0; c < 4; ++c) {
    std::vector<unsigned char> a(64 * 32), b(64 * 32);
    std::vector<int> sa(64), sb(64);
    for (int i = 0; i < 64 * 32; ++i) {
      a[i] = enc(rand() % 5 - 2);
      b[i] = enc(rand() % 5 - 2);
    }
    for (int l = 0; l < 64; ++l) {
      // case 0: unit scales; 1: random A scales; 2: random B scales; 3: both
      sa[l] = 127 + ((c & 1) ? rand() % 3 : 0);
      sb[l] = 127 + ((c & 2) ? rand() % 3 : 0);
    }
    hipMemcpy(da, a.data(), 64 * 32, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), 64 * 32, hipMemcpyHostToDevice);
    hipMemcpy(dsa, sa.data(), 256, hipMemcpyHostToDevice);
    hipMemcpy(dsb, sb.data(), 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
    std::vector<float> d(256);
    hipMemcpy(d.data(), dd, 1024, hipMemcpyDeviceToHost);
    fwrite(a.data(), 1, 2048, f);
    fwrite(b.data(), 1, 2048, f);
    fwrite(sa.data(), 4, 64, f);
    fwrite(sb.data(), 4, 64, f);
    fwrite(d.data(), 4, 256, f);
  }
  fclose(f);
  printf("wrote %s\n", out);
  return 0;
}
