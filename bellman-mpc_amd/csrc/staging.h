// Host -> device staging for caller-owned (pageable) buffers: a small pool of host threads
// copies each chunk into a pinned ring slot while the DMA engine moves the previous slot to
// HBM, so a drop-in bh_prove call streams its ~0.5 GB witness at PCIe rate instead of the
// runtime's pageable-copy rate, and the prover starts on the first vectors while the others
// are still in flight (prover.rs:206-231 hands create_proof host Vecs).
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <functional>
#include <mutex>

#include "host_pool.h"

namespace bh {

// Pinned ring of SLOTS buffers feeding H2D copies on one stream.
struct H2DRing {
  static constexpr int SLOTS = 4;
  static constexpr size_t SLOT_BYTES = (size_t)16 << 20;
  void* buf[SLOTS] = {};
  hipEvent_t done[SLOTS] = {};
  bool pending[SLOTS] = {};
  int next = 0;
  hipError_t init();
  void release();
  // dst (device) <- src (pageable host), enqueued on st; returns once every chunk is enqueued
  // (the last SLOTS chunks may still be in flight: record an event on st to wait for them)
  hipError_t copy(HostPool& pool, void* dst, const void* src, size_t bytes, hipStream_t st);
};

// Progress of an asynchronous witness upload, for the prover's streams to wait on: stage 1 =
// density maps, inputs and aux enqueued (ev[0] recorded after them), stage 2 = a, b, c
// enqueued (ev[1]; vec[v] right after vector v).  A failed upload ends in stage -1 with its
// status.  on_vector, when set, runs on the uploading thread right after vector v's copies are
// enqueued and vec[v] recorded (bh_prove: that vector's H transforms, stream-ordered behind
// vec[v]); stage 2 is set only after the last call returned, so it then also means "H enqueued".
struct UploadSync {
  std::mutex mu;
  std::condition_variable cv;
  int stage = 0;
  int status = 0;
  hipEvent_t t0 = nullptr;  // recorded on the copy stream before the first copy (timing)
  hipEvent_t ev[2] = {};
  hipEvent_t vec[3] = {};
  std::function<int(int v)> on_vector;
  void set(int s, int st = 0) {
    std::lock_guard<std::mutex> lk(mu);
    stage = s;
    status = st;
    cv.notify_all();
  }
  // block until the upload reached stage s; false if it failed
  bool wait(int s) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return stage >= s || stage < 0; });
    return stage >= s;
  }
};

}  // namespace bh
