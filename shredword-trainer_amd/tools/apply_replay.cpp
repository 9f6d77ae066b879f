// Host half of the merge loop replayed without a device: reads a SHREDWORD_APPLY_CAPTURE file
// (the initial pair counts and every merge's delta records of one train()), and runs the exact
// selector on it -- select, the guess of the next merge, combine + order, info walk + pushes --
// checking that every select picks the captured merge, and timing each part per merge range.
//
//   g++ -O3 -std=c++17 -march=native -o apply_replay shredword-trainer_amd/tools/apply_replay.cpp \
//       shredword-trainer_amd/csrc/host/selector.cpp -Ishredword-trainer_amd/csrc/host
//   ./apply_replay capture.bin [reps]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "selector.h"

using namespace shred;

struct Merge {
  int32_t a, b, X;
  size_t off, n;
};

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: apply_replay capture.bin [reps]\n");
    return 2;
  }
  const int reps = argc > 2 ? std::atoi(argv[2]) : 3;
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  int64_t hdr[2] = {0, 0};
  std::vector<PairCount> pairs;
  std::vector<DeltaRecord> recs;
  std::vector<Merge> merges;
  char tag;
  while (std::fread(&tag, 1, 1, f) == 1) {
    if (tag == 'R') {
      if (std::fread(hdr, 8, 2, f) != 2) return 3;
    } else if (tag == 'P') {
      uint64_t n;
      if (std::fread(&n, 8, 1, f) != 1) return 3;
      const size_t o = pairs.size();
      pairs.resize(o + n);
      if (std::fread(pairs.data() + o, sizeof(PairCount), n, f) != n) return 3;
    } else if (tag == 'M') {
      int32_t h[3];
      uint64_t n;
      if (std::fread(h, 4, 3, f) != 3 || std::fread(&n, 8, 1, f) != 1) return 3;
      const size_t o = recs.size();
      recs.resize(o + n);
      if (std::fread(recs.data() + o, sizeof(DeltaRecord), n, f) != n) return 3;
      merges.push_back({h[0], h[1], h[2], o, n});
    } else {
      std::fprintf(stderr, "bad tag %d\n", tag);
      return 3;
    }
  }
  std::fclose(f);
  std::fprintf(stderr, "unk %lld min %lld pairs %zu merges %zu records %zu\n", (long long)hdr[0], (long long)hdr[1],
               pairs.size(), merges.size(), recs.size());
  static const size_t edges[] = {0, 1117, 2000, 3500, 5657, 8000, 16000, 24000, 1u << 30};
  const int nb = sizeof(edges) / sizeof(edges[0]) - 1;
  std::printf("{\"merges\": %zu, \"records\": %zu, \"reps\": [", merges.size(), recs.size());
  for (int r = 0; r < reps; ++r) {
    Selector sel;
    sel.reset((int32_t)hdr[0], (uint64_t)hdr[1]);
    sel.add_counts(pairs);
    std::vector<double> ts(nb), tg(nb), tc(nb), tf(nb);
    size_t bad = 0;
    for (size_t i = 0; i < merges.size(); ++i) {
      const Merge& m = merges[i];
      int b = 0;
      while (m.X >= 0 && i >= edges[b + 1]) ++b;
      const double t0 = now_us();
      int32_t a, bb;
      uint64_t fq;
      if (!sel.select(&a, &bb, &fq)) break;
      const double t1 = now_us();
      if (a != m.a || bb != m.b) ++bad;
      const int32_t used[2] = {a, bb};
      int32_t ga, gb;
      sel.predict_avoid(used, 2, 64, &ga, &gb);
      const double t2 = now_us();
      sel.apply_combine(m.a, m.b, m.X, recs.data() + m.off, m.n);
      const double t3 = now_us();
      sel.apply_finish(m.a, m.b, m.X);
      const double t4 = now_us();
      ts[b] += t1 - t0;
      tg[b] += t2 - t1;
      tc[b] += t3 - t2;
      tf[b] += t4 - t3;
    }
    const Selector::Counters& c = sel.counters();
    std::printf("%s{\"mismatched_selects\": %zu, \"cyc\": {\"combine\": %llu, \"order\": %llu, \"walk\": %llu, \"push\": %llu}, "
                "\"ranges_ms\": [",
                r ? ", " : "", bad, (unsigned long long)c.cyc_combine, (unsigned long long)c.cyc_order,
                (unsigned long long)c.cyc_walk, (unsigned long long)c.cyc_push);
    double tot = 0;
    for (int k = 0; k < nb; ++k) {
      std::printf("%s{\"from\": %zu, \"select\": %.2f, \"guess\": %.2f, \"combine\": %.2f, \"finish\": %.2f}", k ? ", " : "",
                  edges[k], ts[k] / 1e3, tg[k] / 1e3, tc[k] / 1e3, tf[k] / 1e3);
      tot += ts[k] + tg[k] + tc[k] + tf[k];
    }
    std::printf("], \"total_ms\": %.2f}", tot / 1e3);
    std::fflush(stdout);
  }
  std::printf("]}\n");
  return 0;
}
