// Host-only stress of bh::HostPool (bellman-mpc_amd/csrc/host_pool.cpp), built by
// tests/test_host_pool.py with g++ (optionally -fsanitize=thread).  Back-to-back parallel_for
// generations with distinct functions, the pattern H2DRing::copy runs once per 16 MB slot:
// every index of every generation must run exactly once, with that generation's function.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "host_pool.h"

int main(int argc, char** argv) {
  const int gens = argc > 1 ? atoi(argv[1]) : 20000;
  const int workers = argc > 2 ? atoi(argv[2]) : 7;
  bh::HostPool pool(workers);
  std::vector<std::atomic<int>> hits(64);
  long bad = 0;
  for (int g = 0; g < gens; g++) {
    const int n = 1 + (g * 7919) % 37;  // 1..37 pieces, some generations run on the caller alone
    for (int i = 0; i < n; i++) hits[i].store(0);
    std::atomic<int> wrong{0};
    const int tag = g;
    std::function<void(int)> fn = [&, tag](int i) {
      if (tag != g || i < 0 || i >= n) wrong.fetch_add(1);
      else hits[i].fetch_add(1);
    };
    pool.parallel_for(n, fn);
    for (int i = 0; i < n; i++) bad += hits[i].load() != 1;
    bad += wrong.load();
  }
  printf("generations %d workers %d bad %ld\n", gens, workers, bad);
  return bad == 0 ? 0 : 1;
}
