// Selector replay benchmark (test-only): drives the product Selector through a recorded merge
// stream -- the initial pair counts and every merge's delta records, written by the CPU harness
// with HH_RECORD=<file> -- and times select() and apply() alone, with nothing else touching the
// caches (as on the GPU box, where the host spins on a flag between merges).  Every selection is
// checked against the recorded merge, so a faster selector that changed the order fails here.
//   selector_replay <record file> <min_pair_freq> [unk_id] [reps]
#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "selector.h"

using namespace shred;

struct Merge { int32_t a, b, X; size_t off, n; };

// The pairs one merge's records change (the combine's keying, selector.cpp apply_combine).
static std::vector<std::pair<int32_t, int32_t>> changed_pairs(const Merge& m, const DeltaRecord* r, int32_t unk) {
  std::vector<std::pair<int32_t, int32_t>> out;
  for (size_t i = 0; i < m.n; ++i) {
    const uint32_t cat = r[i].key & 3u, slot = r[i].key >> 2;
    const int32_t id = slot == 0 ? unk : (int32_t)(slot - 1);
    switch (cat) {
      case kOldLeft: out.push_back({id, m.a}); break;
      case kNewLeft: out.push_back({id, m.X}); break;
      case kOldRight: out.push_back({m.b, id}); break;
      default: out.push_back({m.X, id}); break;
    }
  }
  return out;
}

// reps < 0: the engine's depth-1 guess (predict_next over 256 heap slots, then the late
// correction) replayed against the recorded merges, with each miss classified.
static int classify(const std::vector<PairCount>& pairs, const std::vector<Merge>& merges,
                    const std::vector<DeltaRecord>& recs, uint64_t mpf, int32_t unk) {
  Selector sel;
  sel.reset(unk, mpf);
  sel.add_counts(pairs);
  if (const char* e = std::getenv("SIM")) sel.set_simulate_pops(std::atoi(e) != 0);
  double tp = 0;
  const auto l0 = std::chrono::steady_clock::now();
  const size_t edges[] = {0, 1500, 5657, 16000, (size_t)-1};
  uint64_t hit[4] = {}, cnt[4] = {}, c_new[4] = {}, c_tie[4] = {}, c_chg[4] = {}, c_gdrop[4] = {}, c_other[4] = {};
  int32_t ga = INT32_MIN, gb = INT32_MIN;
  uint64_t gf_pred = 0;
  for (size_t m = 0; m < merges.size(); ++m) {
    int32_t a, b;
    uint64_t fq;
    if (!sel.select(&a, &b, &fq) || a != merges[m].a || b != merges[m].b) return 1;
    int k = 0;
    while (m >= edges[k + 1]) ++k;
    if (m > 0 && ga != INT32_MIN) {
      ++cnt[k];
      if (ga == a && gb == b) {
        ++hit[k];
      } else {
        const Merge& pm = merges[m - 1];
        bool chg = false, gdrop = false;
        for (auto& pr : changed_pairs(pm, recs.data() + pm.off, unk)) {
          chg |= pr.first == a && pr.second == b;
          gdrop |= pr.first == ga && pr.second == gb;
        }
        uint64_t gf = 0;
        uint32_t gv = 0;
        sel.lookup(ga, gb, &gf, &gv);
        if (a == pm.X || b == pm.X) ++c_new[k];
        else if (gf == fq) ++c_tie[k];
        else if (gdrop) ++c_gdrop[k];
        else if (chg) ++c_chg[k];
        else ++c_other[k];
      }
    }
    ga = gb = INT32_MIN;
    int32_t pa, pb;
    const auto p0 = std::chrono::steady_clock::now();
    const bool got = sel.predict_next(a, b, 256, &pa, &pb);
    tp += std::chrono::duration<double>(std::chrono::steady_clock::now() - p0).count();
    if (got) {
      ga = pa;
      gb = pb;
      uint32_t v;
      sel.lookup(ga, gb, &gf_pred, &v);
    }
    sel.apply_combine(a, b, merges[m].X, recs.data() + merges[m].off, merges[m].n);
    uint64_t pf;
    if (ga != INT32_MIN && sel.predict_after(merges[m].X, gf_pred, &pa, &pb, &pf)) {
      ga = pa;
      gb = pb;
    }
    sel.apply_finish(a, b, merges[m].X);
  }
  std::printf("predict %.3f us per merge, whole loop %.3f us per merge\n", 1e6 * tp / (double)merges.size(),
              1e6 * std::chrono::duration<double>(std::chrono::steady_clock::now() - l0).count() / (double)merges.size());
  for (int k = 0; k < 4; ++k)
    std::printf("merges from %zu: guesses %llu hit %.1f%%; misses: new pair %llu, tie %llu, guess dropped %llu, "
                "actual changed %llu, other %llu\n", edges[k], (unsigned long long)cnt[k], 100.0 * hit[k] / std::max<uint64_t>(1, cnt[k]),
                (unsigned long long)c_new[k], (unsigned long long)c_tie[k], (unsigned long long)c_gdrop[k],
                (unsigned long long)c_chg[k], (unsigned long long)c_other[k]);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <record> <min_pair_freq> [unk_id] [reps]\n", argv[0]);
    return 2;
  }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  const uint64_t mpf = std::strtoull(argv[2], nullptr, 10);
  const int32_t unk = argc > 3 ? std::atoi(argv[3]) : 0;
  const int reps = argc > 4 ? std::atoi(argv[4]) : 1;
  uint64_t np = 0;
  if (std::fread(&np, 8, 1, f) != 1) return 2;
  std::vector<PairCount> pairs(np);
  if (std::fread(pairs.data(), sizeof(PairCount), np, f) != np) return 2;
  std::vector<Merge> merges;
  std::vector<DeltaRecord> recs;
  int32_t hdr[4];
  while (std::fread(hdr, 4, 4, f) == 4) {
    const size_t off = recs.size();
    recs.resize(off + (size_t)hdr[3]);
    if (std::fread(recs.data() + off, sizeof(DeltaRecord), (size_t)hdr[3], f) != (size_t)hdr[3]) return 2;
    merges.push_back({hdr[0], hdr[1], hdr[2], off, (size_t)hdr[3]});
  }
  std::fclose(f);
  if (reps < 0) return classify(pairs, merges, recs, mpf, unk);
  using clk = std::chrono::steady_clock;
  Selector sel;
  for (int r = 0; r < reps; ++r) {
    sel.reset(unk, mpf);
    const auto t0 = clk::now();
    sel.add_counts(pairs);
    const auto t1 = clk::now();
    double ts = 0, ta = 0;
    const size_t edges[] = {0, 1500, 5657, 16000, (size_t)-1};
    double rs[4] = {}, ra[4] = {};
    size_t rn[4] = {};
    for (size_t m = 0; m < merges.size(); ++m) {
      int32_t a, b;
      uint64_t fq;
      const auto s0 = clk::now();
      const bool ok = sel.select(&a, &b, &fq);
      const auto s1 = clk::now();
      if (!ok || a != merges[m].a || b != merges[m].b) {
        std::fprintf(stderr, "replay: merge %zu selected (%d,%d), recorded (%d,%d)\n", m, ok ? a : -1, ok ? b : -1,
                     merges[m].a, merges[m].b);
        return 1;
      }
      sel.apply(a, b, merges[m].X, recs.data() + merges[m].off, merges[m].n);
      const auto s2 = clk::now();
      const double ds = std::chrono::duration<double>(s1 - s0).count(), da = std::chrono::duration<double>(s2 - s1).count();
      ts += ds;
      ta += da;
      int k = 0;
      while (m >= edges[k + 1]) ++k;
      rs[k] += ds;
      ra[k] += da;
      rn[k] += 1;
    }
    const auto& c = sel.counters();
    const double M = (double)merges.size();
    std::printf("merges %zu init %.1f ms select %.3f us apply %.3f us per merge (combine %.0f order %.0f walk %.0f "
                "cycles, push %.0f); pops %llu stale %llu pushes %llu records %llu\n",
                merges.size(), 1e3 * std::chrono::duration<double>(t1 - t0).count(), 1e6 * ts / M, 1e6 * ta / M,
                c.cyc_combine / M, c.cyc_order / M, c.cyc_walk / M, c.cyc_push / M, (unsigned long long)c.pops,
                (unsigned long long)c.stale, (unsigned long long)c.pushes, (unsigned long long)c.records);
    for (int k = 0; k < 4; ++k)
      if (rn[k])
        std::printf("  merges from %zu: %zu, select %.2f us apply %.2f us\n", edges[k], rn[k], 1e6 * rs[k] / rn[k],
                    1e6 * ra[k] / rn[k]);
  }
  return 0;
}
