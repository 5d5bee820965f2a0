// Probe: the per-round cost of the cross-workgroup exchange a
// multi-CU furthest point sampling would need.  Each cloud is served by G
// co-resident workgroups; every round each of them publishes a 64-bit
// (distance, index) key with one device-scope atomicMax, counts itself in with
// a release add, waits until all G arrivals of that round are visible
// (acquire, bounded spin), and reads the winning key back -- the minimum
// protocol of one FPS round, with no sweep at all.  Prints us per round for
// G = 2, 4, 8, 16 at 32 clouds (the loss FPS launch: B = 32).
// Cooperative launch guarantees co-residency; every spin is bounded and a
// timeout is reported, so the grid always drains.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void xcu_rounds(unsigned long long *keys, unsigned *cnt, unsigned long long *out, int G, int rounds,
                           int *timeout) {
  const int cloud = blockIdx.x / G, member = blockIdx.x % G;
  unsigned long long acc = 0;
  for (int r = 0; r < rounds; ++r) {
    const int slot = cloud * 2 + (r & 1);
    if (threadIdx.x == 0) {
      // a key that changes per round and member (the sweep's result stand-in)
      const unsigned long long key = ((unsigned long long)((r * 2654435761u) ^ (member * 40503u)) << 20) | member;
      __hip_atomic_fetch_max(&keys[slot * 32 + (r >> 1) % 32], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&cnt[slot], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned want = (unsigned)G * (unsigned)(r / 2 + 1);
      long spins = 0;
      while (__hip_atomic_load(&cnt[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < want) {
        if (++spins > (1l << 24)) {
          atomicExch(timeout, 1);
          break;
        }
      }
      acc += __hip_atomic_load(&keys[slot * 32 + (r >> 1) % 32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();  // the rest of the workgroup waits for the winner, as the sweep would
    if (*(volatile int *)timeout) break;
  }
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

int main() {
  const int clouds = 32, rounds = 2048;
  for (int G : {2, 4, 8, 16}) {
    const int nblk = clouds * G;
    unsigned long long *keys, *out;
    unsigned *cnt;
    int *timeout;
    (void)hipMalloc(&keys, (size_t)clouds * 2 * 32 * 8);
    (void)hipMalloc(&cnt, (size_t)clouds * 2 * 4);
    (void)hipMalloc(&out, (size_t)nblk * 8);
    (void)hipMalloc(&timeout, 4);
    float best = 1e30f;
    int to = 0;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipMemset(keys, 0, (size_t)clouds * 2 * 32 * 8);
      (void)hipMemset(cnt, 0, (size_t)clouds * 2 * 4);
      (void)hipMemset(timeout, 0, 4);
      int G_ = G, rounds_ = rounds;
      void *args[] = {&keys, &cnt, &out, &G_, &rounds_, &timeout};
      hipEvent_t a, b;
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      (void)hipEventRecord(a);
      const hipError_t e = hipLaunchCooperativeKernel((const void *)xcu_rounds, dim3(nblk), dim3(256), args, 0, 0);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      if (e != hipSuccess) {
        printf("G=%d: cooperative launch failed: %s\n", G, hipGetErrorString(e));
        break;
      }
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      (void)hipMemcpy(&to, timeout, 4, hipMemcpyDeviceToHost);
      if (to) break;
      if (ms < best) best = ms;
    }
    if (to)
      printf("G=%d: spin bound hit (not co-resident?)\n", G);
    else
      printf("G=%d workgroups/cloud x %d clouds: %.3f us per round (exchange only, no sweep)\n", G, clouds,
             best * 1000.f / rounds);
    (void)hipFree(keys);
    (void)hipFree(cnt);
    (void)hipFree(out);
    (void)hipFree(timeout);
  }
  return 0;
}
