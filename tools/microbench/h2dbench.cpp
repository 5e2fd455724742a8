// Host -> device upload paths on one MI355X (the drop-in bh_prove's witness upload, staging.h):
//   pageable hipMemcpy, pinned DMA, the library's staging ring at several worker counts and slot
//   sizes, hipHostRegister + DMA (and the registration's own cost), and a stream-ordered gate
//   (hipStreamWaitValue32 on signal memory released by hipStreamWriteValue32 on another stream).
// build: hipcc --offload-arch=gfx950 -O2 -std=c++17 -I../../bellman-mpc_amd/csrc h2dbench.cpp
//        ../../bellman-mpc_amd/csrc/staging.cpp ../../bellman-mpc_amd/csrc/host_pool.cpp -o h2dbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <thread>

#include "host_pool.h"
#include "staging.h"

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void k_mark(volatile uint32_t* p) { *p = 1; }

// a VALU-saturating kernel (every CU, 8 waves per SIMD) for a bounded number of iterations
__global__ void __launch_bounds__(256) k_busy(uint64_t* out, int iters) {
  uint64_t x = threadIdx.x + blockIdx.x, y = x * 3 + 1;
  for (int i = 0; i < iters; i++) {
    x = x * y + 7;
    y = y * x + 11;
  }
  if (x == 0x12345) out[0] = y;
}

int main(int argc, char** argv) {
  const size_t bytes = (size_t)(argc > 1 ? atoi(argv[1]) : 128) << 20;
  CK(hipSetDevice(0));
  uint8_t* host = (uint8_t*)aligned_alloc(4096, bytes);
  for (size_t i = 0; i < bytes; i += 64) host[i] = (uint8_t)i;  // fault every page in
  void* dev;
  CK(hipMalloc(&dev, bytes));
  hipStream_t st, st2;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
  auto rate = [&](double ms) { return bytes / (ms * 1e6); };
  auto best3 = [&](auto fn) {
    double b = 1e30;
    for (int r = 0; r < 4; r++) {
      double t0 = now_ms();
      fn();
      double t = now_ms() - t0;
      if (r && t < b) b = t;
    }
    return b;
  };
  printf("bytes %zu MB, hardware threads %u\n", bytes >> 20, std::thread::hardware_concurrency());
  double t = best3([&] { CK(hipMemcpy(dev, host, bytes, hipMemcpyHostToDevice)); });
  printf("pageable hipMemcpy            %7.2f ms  %6.1f GB/s\n", t, rate(t));
  void* pin;
  CK(hipHostMalloc(&pin, bytes, hipHostMallocDefault));
  memcpy(pin, host, bytes);
  t = best3([&] { CK(hipMemcpyAsync(dev, pin, bytes, hipMemcpyHostToDevice, st)); CK(hipStreamSynchronize(st)); });
  printf("pinned DMA (one copy)         %7.2f ms  %6.1f GB/s\n", t, rate(t));
  for (int workers : {3, 7, 11, 15}) {
    bh::HostPool pool(workers);
    t = best3([&] {
      pool.parallel_for(pool.size(), [&](int i) {
        const size_t piece = bytes / pool.size();
        memcpy((uint8_t*)pin + i * piece, host + i * piece, piece);
      });
    });
    printf("host memcpy -> pinned, %2d thr %7.2f ms  %6.1f GB/s\n", pool.size(), t, rate(t));
    bh::H2DRing ring;
    t = best3([&] { CK(ring.copy(pool, dev, host, bytes, st)); CK(hipStreamSynchronize(st)); });
    printf("staging ring (4 x 16 MB), %2d thr %7.2f ms  %6.1f GB/s\n", pool.size(), t, rate(t));
    ring.release();
  }
  {
    // the same copies while every CU is saturated by a kernel on another stream (the proof's
    // situation: the accumulations hold every SIMD)
    hipStream_t sb;
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    uint64_t* junk;
    CK(hipMalloc(&junk, 64));
    hipEvent_t b0, b1;
    CK(hipEventCreate(&b0));
    CK(hipEventCreate(&b1));
    CK(hipEventRecord(b0, sb));
    k_busy<<<256 * 32, 256, 0, sb>>>(junk, 1 << 14);
    CK(hipEventRecord(b1, sb));
    CK(hipEventSynchronize(b1));
    float bms = 0;
    CK(hipEventElapsedTime(&bms, b0, b1));
    const int iters = (int)((1 << 14) * (400.0 / std::max(bms, 0.01f)));  // ~400 ms
    printf("busy kernel: %.1f ms at 2^14 iterations -> %d iterations\n", bms, iters);
    bh::HostPool pool(7);
    bh::H2DRing ring;
    for (int rep = 0; rep < 2; rep++) {
      k_busy<<<256 * 32, 256, 0, sb>>>(junk, iters);
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
      double ta = now_ms();
      CK(hipMemcpyAsync(dev, pin, bytes, hipMemcpyHostToDevice, st));
      CK(hipStreamSynchronize(st));
      double tp = now_ms() - ta;
      ta = now_ms();
      CK(hipMemcpy(dev, host, bytes, hipMemcpyHostToDevice));
      double tq = now_ms() - ta;
      ta = now_ms();
      CK(ring.copy(pool, dev, host, bytes, st));
      CK(hipStreamSynchronize(st));
      double tr = now_ms() - ta;
      const bool busy = hipStreamQuery(sb) == hipErrorNotReady;
      printf("under a busy GPU (still busy after: %d): pinned DMA %.2f ms %.1f GB/s, pageable %.2f ms %.1f GB/s, "
             "ring %.2f ms %.1f GB/s\n", (int)busy, tp, rate(tp), tq, rate(tq), tr, rate(tr));
      CK(hipStreamSynchronize(sb));
    }
    ring.release();
  }
  double t0 = now_ms();
  CK(hipHostRegister(host, bytes, hipHostRegisterDefault));
  double treg = now_ms() - t0;
  t = best3([&] { CK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, st)); CK(hipStreamSynchronize(st)); });
  t0 = now_ms();
  CK(hipHostUnregister(host));
  double tun = now_ms() - t0;
  printf("hipHostRegister %7.2f ms, DMA %7.2f ms %6.1f GB/s, unregister %7.2f ms\n", treg, t, rate(t), tun);

  // stream-ordered gate: st2 waits on a 32-bit value that st writes later
  int can = 0;
  (void)hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0);
  printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", can);
  uint32_t* sig = nullptr;
  hipError_t e = hipExtMallocWithFlags((void**)&sig, 8, hipMallocSignalMemory);
  printf("hipExtMallocWithFlags(hipMallocSignalMemory) -> %s\n", hipGetErrorString(e));
  if (e == hipSuccess) {
    uint32_t* mark;
    CK(hipHostMalloc(&mark, 64, hipHostMallocCoherent));
    *(volatile uint32_t*)mark = 0;
    CK(hipMemsetAsync(sig, 0, 8, st));
    CK(hipStreamSynchronize(st));
    hipEvent_t done;
    CK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    for (uint32_t gen = 1; gen <= 3; gen++) {
      *(volatile uint32_t*)mark = 0;
      e = hipStreamWaitValue32(st2, sig, gen, hipStreamWaitValueGte, 0xffffffffu);
      if (e != hipSuccess) { printf("hipStreamWaitValue32 -> %s\n", hipGetErrorString(e)); break; }
      k_mark<<<1, 1, 0, st2>>>(mark);
      CK(hipEventRecord(done, st2));
      std::this_thread::sleep_for(std::chrono::milliseconds(30));
      const bool early = *(volatile uint32_t*)mark != 0 || hipEventQuery(done) == hipSuccess;
      const double tw = now_ms();
      CK(hipStreamWriteValue32(st, sig, gen, 0));
      CK(hipEventSynchronize(done));
      printf("gate gen %u: ran before release %d, released -> done in %.3f ms, mark %u\n", gen, (int)early,
             now_ms() - tw, *(volatile uint32_t*)mark);
    }
    CK(hipStreamSynchronize(st));
    CK(hipStreamSynchronize(st2));
  }
  CK(hipDeviceSynchronize());
  printf("ok\n");
  return 0;
}
