// HBM streaming probe: which launch/access structure reaches the highest bf16 copy-like
// bandwidth on MI355X (drives the design of the element-wise fake-quant kernels).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef unsigned int V __attribute__((ext_vector_type(4)));
__device__ __forceinline__ V xf(V v) { v.x ^= 0x00010001u; v.y ^= 0x00010001u; v.z ^= 1u; v.w ^= 1u; return v; }

template <int U> __global__ __launch_bounds__(256) void gs(const V* __restrict__ x, V* __restrict__ y, long n) {
  long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    V v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) y[i + u * stride] = xf(v[u]);
  }
  for (; i < n; i += stride) y[i] = xf(x[i]);
}
// contiguous chunk per block: block b handles [b*256*U, (b+1)*256*U)
template <int U, bool NT> __global__ __launch_bounds__(256) void chunk(const V* __restrict__ x, V* __restrict__ y, long n) {
  long base = (long)blockIdx.x * 256 * U + threadIdx.x;
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { long i = base + u * 256; if (i < n) v[u] = NT ? __builtin_nontemporal_load(x + i) : x[i]; }
#pragma unroll
  for (int u = 0; u < U; ++u) { long i = base + u * 256; if (i < n) { if (NT) __builtin_nontemporal_store(xf(v[u]), y + i); else y[i] = xf(v[u]); } }
}
// persistent chunks: grid-stride over chunks of 256*U vectors
template <int U> __global__ __launch_bounds__(256) void pchunk(const V* __restrict__ x, V* __restrict__ y, long n) {
  long nch = (n + 256L * U - 1) / (256L * U);
  for (long c = blockIdx.x; c < nch; c += gridDim.x) {
    long base = c * 256 * U + threadIdx.x;
    V v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { long i = base + u * 256; if (i < n) v[u] = x[i]; }
#pragma unroll
    for (int u = 0; u < U; ++u) { long i = base + u * 256; if (i < n) y[i] = xf(v[u]); }
  }
}
__global__ void rd(const V* __restrict__ x, long n, unsigned* out) {
  long stride = (long)gridDim.x * 256; unsigned m = 0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) { V v = x[i]; m = max(m, max(max((unsigned)v.x, (unsigned)v.y), max((unsigned)v.z, (unsigned)v.w))); }
  if (m == 0x12345678u) out[0] = m;
}

int main() {
  const long bytes = 256L << 20, n = bytes / 16;
  const int NB = 4;
  std::vector<V*> xs(NB), ys(NB);
  for (int b = 0; b < NB; ++b) { CK(hipMalloc(&xs[b], bytes)); CK(hipMalloc(&ys[b], bytes)); CK(hipMemset(xs[b], 1, bytes)); }
  unsigned* o; CK(hipMalloc(&o, 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch, double traffic) {
    for (int w = 0; w < 8; ++w) launch(w % NB);
    CK(hipDeviceSynchronize());
    const int it = 40;
    CK(hipEventRecord(e0));
    for (int w = 0; w < it; ++w) launch(w % NB);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= it;
    printf("%-28s %8.4f ms  %7.1f GB/s\n", name, ms, traffic / (ms * 1e-3) / 1e9);
    return 0;
  };
  double t2 = 2.0 * bytes;
  for (int g : {1024, 2048, 4096}) {
    char nm[64];
    snprintf(nm, 64, "gs1 grid=%d", g); run(nm, [&](int b) { gs<1><<<g, 256>>>(xs[b], ys[b], n); }, t2);
    snprintf(nm, 64, "gs2 grid=%d", g); run(nm, [&](int b) { gs<2><<<g, 256>>>(xs[b], ys[b], n); }, t2);
    snprintf(nm, 64, "gs4 grid=%d", g); run(nm, [&](int b) { gs<4><<<g, 256>>>(xs[b], ys[b], n); }, t2);
    snprintf(nm, 64, "pchunk4 grid=%d", g); run(nm, [&](int b) { pchunk<4><<<g, 256>>>(xs[b], ys[b], n); }, t2);
    snprintf(nm, 64, "pchunk8 grid=%d", g); run(nm, [&](int b) { pchunk<8><<<g, 256>>>(xs[b], ys[b], n); }, t2);
  }
  run("chunk1 (1 vec/thread)", [&](int b) { chunk<1, false><<<(n + 255) / 256, 256>>>(xs[b], ys[b], n); }, t2);
  run("chunk2", [&](int b) { chunk<2, false><<<(n + 511) / 512, 256>>>(xs[b], ys[b], n); }, t2);
  run("chunk4", [&](int b) { chunk<4, false><<<(n + 1023) / 1024, 256>>>(xs[b], ys[b], n); }, t2);
  run("chunk8", [&](int b) { chunk<8, false><<<(n + 2047) / 2048, 256>>>(xs[b], ys[b], n); }, t2);
  run("chunk4 nt", [&](int b) { chunk<4, true><<<(n + 1023) / 1024, 256>>>(xs[b], ys[b], n); }, t2);
  run("chunk8 nt", [&](int b) { chunk<8, true><<<(n + 2047) / 2048, 256>>>(xs[b], ys[b], n); }, t2);
  run("read-only gs grid=2048", [&](int b) { rd<<<2048, 256>>>(xs[b], n, o); }, (double)bytes);
  run("read-only gs grid=8192", [&](int b) { rd<<<8192, 256>>>(xs[b], n, o); }, (double)bytes);
  run("hipMemcpyAsync D2D", [&](int b) { (void)hipMemcpyAsync(ys[b], xs[b], bytes, hipMemcpyDeviceToDevice); }, t2);
  return 0;
}
