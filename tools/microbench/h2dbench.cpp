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
  hipError_t e = hipExtMallocWithFlags((void**)&sig, 64, hipMallocSignalMemory);
  printf("hipExtMallocWithFlags(hipMallocSignalMemory) -> %s\n", hipGetErrorString(e));
  if (e == hipSuccess) {
    uint32_t* mark;
    CK(hipHostMalloc(&mark, 64, hipHostMallocCoherent));
    *(volatile uint32_t*)mark = 0;
    CK(hipMemsetAsync(sig, 0, 64, st));
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
