// Pinned staging for host -> device copies of caller buffers (see staging.h).
#include "staging.h"

#include <string.h>

#include <algorithm>

namespace bh {

hipError_t H2DRing::init() {
  if (buf[0]) return hipSuccess;
  for (int k = 0; k < SLOTS; k++) {
    hipError_t e = hipHostMalloc(&buf[k], SLOT_BYTES, hipHostMallocDefault);
    if (e != hipSuccess) return e;
    e = hipEventCreateWithFlags(&done[k], hipEventDisableTiming);
    if (e != hipSuccess) return e;
    pending[k] = false;
  }
  return hipSuccess;
}

void H2DRing::release() {
  for (int k = 0; k < SLOTS; k++) {
    if (pending[k] && done[k]) (void)hipEventSynchronize(done[k]);
    if (buf[k]) (void)hipHostFree(buf[k]);
    if (done[k]) (void)hipEventDestroy(done[k]);
    buf[k] = nullptr;
    done[k] = nullptr;
    pending[k] = false;
  }
}

hipError_t H2DRing::copy(HostPool& pool, void* dst, const void* src, size_t bytes, hipStream_t st) {
  hipError_t e = init();
  if (e != hipSuccess) return e;
  const uint8_t* s = static_cast<const uint8_t*>(src);
  uint8_t* d = static_cast<uint8_t*>(dst);
  for (size_t off = 0; off < bytes; off += SLOT_BYTES) {
    const size_t len = std::min(SLOT_BYTES, bytes - off);
    const int k = next;
    next = (next + 1) % SLOTS;
    if (pending[k] && (e = hipEventSynchronize(done[k])) != hipSuccess) return e;  // slot's last DMA done
    uint8_t* slot = static_cast<uint8_t*>(buf[k]);
    const int parts = std::max(1, std::min(pool.size() * 2, (int)(len >> 20)));  // >= 1 MB per piece
    const size_t piece = (len + parts - 1) / parts;
    pool.parallel_for(parts, [&](int i) {
      const size_t a = (size_t)i * piece, b = std::min(len, a + piece);
      if (a < b) memcpy(slot + a, s + off + a, b - a);
    });
    if ((e = hipMemcpyAsync(d + off, slot, len, hipMemcpyHostToDevice, st)) != hipSuccess) return e;
    if ((e = hipEventRecord(done[k], st)) != hipSuccess) return e;
    pending[k] = true;
  }
  return hipSuccess;
}

}  // namespace bh
