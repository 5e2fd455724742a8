// A kernel's identity for the scratch-budget check (scratch.cpp): each translation unit lists the
// kernels it emits with the block size and dynamic LDS they launch with.
#pragma once
#include <stddef.h>

#include <vector>

namespace bh {
struct KernInfo {
  const char* name;
  const void* fn;
  int block;
  size_t lds;
};
}  // namespace bh
