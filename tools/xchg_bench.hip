// Microbenchmark: inter-workgroup ping-pong latency on gfx950 for the exchange protocols the
// fused update kernel could use between the workgroups of one policy (blocks b and b + 8,
// expected on the same XCD).  Also prints each block's XCC / CU placement.
//
//   hipcc --offload-arch=gfx950 -O3 tools/xchg_bench.hip -o tools/xchg_bench && tools/xchg_bench
//
// Protocol p (template): how the ping writer stores and how the poller loads one 8-byte
// {value, tag} granule.  A round trip = block 0 writes tag t, block 8 sees it and writes t,
// block 0 sees it.  Each poll is bounded (timeout -> reported as failure, never a hang).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned v2u __attribute__((ext_vector_type(2)));

template <int P>
__device__ __forceinline__ void put(unsigned long long* g, unsigned tag) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(g, 0, 8, 0x00020000);
  const v2u x = {tag, tag};
  if constexpr (P == 0) __builtin_amdgcn_raw_buffer_store_b64(x, r, 0, 0, 16);        // sc1
  else if constexpr (P == 1) __builtin_amdgcn_raw_buffer_store_b64(x, r, 0, 0, 0);    // plain
  else if constexpr (P == 2) __builtin_amdgcn_raw_buffer_store_b64(x, r, 0, 0, 0);    // plain
  else if constexpr (P == 3) __hip_atomic_store(g, ((unsigned long long)tag << 32) | tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else if constexpr (P == 4) __builtin_amdgcn_raw_buffer_store_b64(x, r, 0, 0, 1);    // sc0
  else if constexpr (P == 5) __builtin_amdgcn_raw_buffer_store_b64(x, r, 0, 0, 16);   // sc1
  else if constexpr (P == 6) __builtin_amdgcn_raw_buffer_store_b64(x, r, 0, 0, 0);    // plain
  else if constexpr (P == 7) __builtin_amdgcn_raw_buffer_store_b64(x, r, 0, 0, 2);    // nt
}

__device__ unsigned long long g_zero;   // 0 at run time, opaque to the compiler
template <int P>
__device__ __forceinline__ unsigned get(unsigned long long* g) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(g, 0, 8, 0x00020000);
  if constexpr (P == 0) return __builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 16)[1];   // sc1 load
  else if constexpr (P == 1) return __builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 16)[1];
  else if constexpr (P == 2) {                                                           // scalar, glc
    unsigned long long v;
    asm volatile("s_load_dwordx2 %0, %1, 0x0 glc\n s_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(g) : "memory");
    return (unsigned)(v >> 32);
  } else if constexpr (P == 3) return (unsigned)(__hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32);
  else if constexpr (P == 4) return __builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 1)[1];  // sc0 load
  else if constexpr (P == 5) {                                                             // inv sc1 + plain
    asm volatile("buffer_inv sc1" ::: "memory");
    return __builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0)[1];
  } else if constexpr (P == 6) {                                                           // atomic or 0
    return (unsigned)(__hip_atomic_fetch_add(g, g_zero, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >> 32);
  } else {
    return __builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 2)[1];                          // nt load
  }
}

template <int P>
__global__ void k_pingpong(unsigned long long* box, int rounds, unsigned* place, unsigned long long* out) {
  unsigned xcc, hwid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  if (threadIdx.x == 0) { place[2 * blockIdx.x] = xcc; place[2 * blockIdx.x + 1] = hwid; }
  const int b = blockIdx.x;
  if (!(b == 0 || b == 8) || threadIdx.x != 0) return;
  unsigned long long* mine = box + (b == 0 ? 0 : 8);
  unsigned long long* other = box + (b == 0 ? 8 : 0);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int ok = 1;
  for (int i = 1; i <= rounds && ok; ++i) {
    if (b == 0) put<P>(mine, (unsigned)i);
    const unsigned long long ts = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      asm volatile("" ::: "memory");   // every poll is a fresh load
      if (get<P>(other) == (unsigned)i) break;
      if (__builtin_amdgcn_s_memrealtime() - ts > 20000000ull) { ok = 0; break; }   // 200 ms
    }
    if (b == 8) put<P>(mine, (unsigned)i);
  }
  if (b == 0) { out[0] = __builtin_amdgcn_s_memrealtime() - t0; out[1] = ok; }
}

template <int P>
static void run(const char* name, unsigned long long* box, unsigned* place, unsigned long long* out, bool show) {
  const int rounds = 2000;
  (void)hipMemset(box, 0, 4096);
  (void)hipMemset(out, 0, 16);
  hipLaunchKernelGGL(k_pingpong<P>, dim3(28), dim3(256), 0, 0, box, rounds, place, out);
  (void)hipDeviceSynchronize();
  unsigned long long h[2];
  unsigned pl[56];
  (void)hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
  (void)hipMemcpy(pl, place, sizeof(pl), hipMemcpyDeviceToHost);
  printf("%-34s %s  round trip %.3f us\n", name, h[1] ? "ok  " : "FAIL", h[0] * 0.01 / rounds);
  if (show) {
    for (int i = 0; i < 28; ++i)
      printf("  block %2d: xcc %u se %u cu %u\n", i, pl[2 * i] & 0xf, (pl[2 * i + 1] >> 13) & 0x7, (pl[2 * i + 1] >> 8) & 0xf);
  }
}

int main() {
  unsigned long long *box, *out;
  unsigned* place;
  (void)hipMalloc(&box, 4096);
  (void)hipMalloc(&out, 16);
  (void)hipMalloc(&place, 56 * sizeof(unsigned));
  run<0>("sc1 store / sc1 load", box, place, out, true);
  run<1>("plain store / sc1 load", box, place, out, false);
  run<2>("plain store / s_load glc", box, place, out, false);
  run<3>("agent atomic store / load", box, place, out, false);
  run<4>("sc0 store / sc0 load", box, place, out, false);
  run<5>("sc1 store / inv sc1 + load", box, place, out, false);
  run<6>("plain store / wg fetch_add 0", box, place, out, false);
  run<7>("nt store / nt load", box, place, out, false);
  return 0;
}
