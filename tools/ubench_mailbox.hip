// What a stream-service call costs, piece by piece: one persistent wave polls a
// pinned, coherent, device-mapped host mailbox, as k_stream_service does, and answers N
// requests; the host times the round trips.  Variants:
//   0  poll seq, then set ack (release, system scope)                 -> the bare ping-pong
//   1  + read the first 4 KiB of the mailbox in one burst              -> + the request read
//   2  + write 128 B of results back to the mailbox before the ack     -> a service call's shape
//   3  as 2, the ack a relaxed store after the wave's stores are done  -> what the release costs
//   4  as 2, polling with s_sleep 0 instead of 1
//   5  as 2, with seq and the request in fine-grained device memory the host writes through the
//      BAR (the ack and results still in host memory); its own JSON line, after the others
//   6  as 2, polling with relaxed loads (no cache invalidate per poll) and one acquire fence
//      after the request is seen
//   7  as 6, with four polls in flight (a new load issued as the oldest is checked)
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_mailbox tools/ubench_mailbox.hip
//   tools/ubench_mailbox [n]   -> one JSON line, microseconds per call
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef unsigned int u32;
typedef unsigned long long u64;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

struct alignas(64) Box {
  u32 seq, p0[15];
  u32 ack, p1[15];
  u32 stop, p2[15];
  u32 pad[16];
};

__device__ __forceinline__ u32 acq(const u32* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ u32 rlx(const u32* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int V>
__global__ __launch_bounds__(64) void k_mailbox(Box* box, Box* resp, u32 n, u32* sink) {
  char* const h = (char*)box;
  char* const hr = (char*)resp;
  const u32 lane = threadIdx.x;
  u32 acc = 0;
  for (u32 i = 1; i <= n; ++i) {
    u64 polls = 0;
    if (V == 7) {
      u32 a0 = rlx(&box->seq);
      __builtin_amdgcn_s_sleep(1);
      u32 a1 = rlx(&box->seq);
      __builtin_amdgcn_s_sleep(1);
      u32 a2 = rlx(&box->seq);
      __builtin_amdgcn_s_sleep(1);
      u32 a3 = rlx(&box->seq);
      for (;;) {
        if (__builtin_amdgcn_readfirstlane(a0) == i) break;
        a0 = rlx(&box->seq);
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_readfirstlane(a1) == i) break;
        a1 = rlx(&box->seq);
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_readfirstlane(a2) == i) break;
        a2 = rlx(&box->seq);
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_readfirstlane(a3) == i) break;
        a3 = rlx(&box->seq);
        __builtin_amdgcn_s_sleep(1);
        if ((++polls & 15) == 0 &&
            (polls > (1ull << 20) || __builtin_amdgcn_readfirstlane(rlx(&box->stop)))) {
          sink[0] = 0xDEAD;
          return;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    for (; V != 7;) {
      const u32 s = __builtin_amdgcn_readfirstlane(V == 6 ? rlx(&box->seq) : acq(&box->seq));
      if (V == 6 && s == i) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      if (s == i) break;
      if (++polls > (1ull << 22) || __builtin_amdgcn_readfirstlane(acq(&box->stop))) {
        sink[0] = 0xDEAD;  // (the host gave up: leave)
        return;
      }
      if (V == 4) __builtin_amdgcn_s_sleep(0);
      else __builtin_amdgcn_s_sleep(1);
    }
    if (V >= 1) {
      u32x4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = *(const u32x4*)(h + 256 + 16 * (lane + 64 * j));
#pragma unroll
      for (int j = 0; j < 4; ++j) acc += v[j].x ^ v[j].w;
    }
    if (V >= 2 && lane < 8) {
      u32x4 r = {i, acc, lane, 0};
      *(u32x4*)(hr + 8192 + 16 * lane) = r;
    }
    if (V == 3) {
      __builtin_amdgcn_s_waitcnt(0);
      if (lane == 0) __hip_atomic_store(&resp->ack, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (lane == 0) {
      __hip_atomic_store(&resp->ack, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if (lane == 0) sink[0] = acc;
}

// hb / db: the request side (host and device addresses); hr / dr: the response side
template <int V>
static double run(Box* hb, Box* db, Box* hr, Box* dr, u32* sink, u32 n) {
  memset(hb, 0, sizeof(Box));
  memset(hr, 0, sizeof(Box));
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipLaunchKernelGGL(k_mailbox<V>, dim3(1), dim3(64), 0, s, db, dr, n, sink);
  double t0 = 0;
  for (u32 i = 1; i <= n; ++i) {
    if (i == 65) t0 = std::chrono::duration<double, std::micro>(
                          std::chrono::steady_clock::now().time_since_epoch()).count();
    memset((char*)hb + 256, (int)i, 2048);  // a request block's worth of stores
    __atomic_store_n(&hb->seq, i, __ATOMIC_RELEASE);
    if (V == 5) __builtin_ia32_sfence();  // (write-combined BAR stores: push them out)
    const auto w0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(&hr->ack, __ATOMIC_ACQUIRE) != i) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() - w0 > std::chrono::seconds(5)) {
        __atomic_store_n(&hb->stop, 1u, __ATOMIC_RELEASE);
        (void)hipStreamSynchronize(s);
        fprintf(stderr, "variant %d: no answer at request %u\n", V, i);
        exit(1);
      }
    }
  }
  const double t1 = std::chrono::duration<double, std::micro>(
                        std::chrono::steady_clock::now().time_since_epoch()).count();
  (void)hipStreamSynchronize(s);
  (void)hipStreamDestroy(s);
  return (t1 - t0) / (n - 64);
}

int main(int argc, char** argv) {
  const u32 n = argc > 1 ? (u32)atoi(argv[1]) : 20000;
  void* hb = nullptr;
  if (hipHostMalloc(&hb, 16384, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
  void* db = nullptr;
  (void)hipHostGetDevicePointer(&db, hb, 0);
  u32* sink = nullptr;
  (void)hipMalloc((void**)&sink, 64);
  Box *H = (Box*)hb, *D = (Box*)db;
  const double v0 = run<0>(H, D, H, D, sink, n), v1 = run<1>(H, D, H, D, sink, n);
  const double v2 = run<2>(H, D, H, D, sink, n), v3 = run<3>(H, D, H, D, sink, n);
  const double v4 = run<4>(H, D, H, D, sink, n);
  const double v6 = run<6>(H, D, H, D, sink, n), v7 = run<7>(H, D, H, D, sink, n);
  printf("{\"n\": %u, \"pingpong_us\": %.3f, \"burst_read_us\": %.3f, \"write_back_us\": %.3f, "
         "\"relaxed_ack_us\": %.3f, \"sleep0_us\": %.3f, \"relaxed_poll_us\": %.3f, "
         "\"four_polls_in_flight_us\": %.3f}\n", n, v0, v1, v2, v3, v4, v6, v7);
  fflush(stdout);
  if (argc > 2 && !strcmp(argv[2], "vram")) {
    void* vb = nullptr;
    if (hipExtMallocWithFlags(&vb, 16384, hipDeviceMallocFinegrained) != hipSuccess) {
      printf("{\"vram\": \"hipExtMallocWithFlags failed\"}\n");
      return 0;
    }
    hipPointerAttribute_t at;
    (void)hipPointerGetAttributes(&at, vb);
    printf("{\"vram_host_pointer\": \"%p\", \"vram_device_pointer\": \"%p\"}\n", at.hostPointer,
           at.devicePointer);
    fflush(stdout);
    if (!at.hostPointer) return 0;
    const double v5 = run<5>((Box*)at.hostPointer, (Box*)vb, H, D, sink, n);
    printf("{\"n\": %u, \"vram_request_us\": %.3f}\n", n, v5);
  }
  return 0;
}
