// gen_corpus — deterministic synthetic corpus generator for the BPE path.
//
// Implements SURVEY.md §8 d2: word types are drawn from a Zipf(1.1) distribution over a
// Heaps-law-growing universe (U(n) = 30 * n^0.55 types after n tokens), each type's spelling
// is a pure function of (seed, type id): length 1 + Geometric(0.2) capped at 20 characters,
// letters Zipf(1.1) over the type's script alphabet.  12 words per line, ' ' and '\n'.
//
// Output is a pure function of (bytes, seed, script): the stream is produced in fixed blocks of
// LINES_PER_BLOCK lines, each block seeded from (seed, block index), so the thread count never
// changes a byte.  The file is exactly `bytes` long and its last byte is '\n'.
//
//   gen_corpus --bytes N --seed S --script ascii|utf8|mixed --out PATH [--threads T]
//
// This is benchmark / test infrastructure: the reference ships no corpus generator
// (SURVEY.md §4, §6), so every config's corpus comes from here.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr int kWordsPerLine = 12;
constexpr int kLinesPerBlock = 4096;
constexpr int kMaxChars = 20;

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct Rng {  // xoshiro256**
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    for (int i = 0; i < 4; ++i) { seed = splitmix64(seed); s[i] = seed; }
  }
  static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  inline uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
    s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  inline double uniform() { return (double)(next() >> 11) * 0x1.0p-53; }
};

// Rejection-inversion sampling of Zipf(exponent) over {1..n} (Hörmann & Derflinger 1996).
struct Zipf {
  double e, hx1, hn, s;
  uint64_t n;
  static double helper1(double x) { return std::fabs(x) > 1e-8 ? std::log1p(x) / x : 1.0 - x * (0.5 - x * (1.0 / 3.0 - 0.25 * x)); }
  static double helper2(double x) { return std::fabs(x) > 1e-8 ? std::expm1(x) / x : 1.0 + x * 0.5 * (1.0 + x * (1.0 / 3.0) * (1.0 + 0.25 * x)); }
  double h(double x) const { return std::exp(-e * std::log(x)); }
  double hint(double x) const { const double lx = std::log(x); return helper2((1.0 - e) * lx) * lx; }
  double hinv(double x) const {
    double t = x * (1.0 - e);
    if (t < -1.0) t = -1.0;
    return std::exp(helper1(t) * x);
  }
  Zipf(uint64_t n_, double e_) : e(e_), n(n_) {
    hx1 = hint(1.5) - 1.0;
    hn = hint((double)n + 0.5);
    s = 2.0 - hinv(hint(2.5) - h(2.0));
  }
  uint64_t sample(Rng& r) const {
    for (;;) {
      const double u = hn + r.uniform() * (hx1 - hn);
      const double x = hinv(u);
      double kd = std::floor(x + 0.5);
      if (kd < 1.0) kd = 1.0;
      if (kd > (double)n) kd = (double)n;
      if (kd - x <= s || u >= hint(kd + 0.5) - h(kd)) return (uint64_t)kd;
    }
  }
};

struct Script {
  std::vector<uint32_t> cps;   // code points in letter-rank order
  std::vector<double> cdf;     // Zipf(1.1) cdf over ranks
};

Script make_script(std::vector<uint32_t> cps) {
  Script s;
  s.cps = std::move(cps);
  double acc = 0.0;
  for (size_t r = 0; r < s.cps.size(); ++r) { acc += std::pow((double)(r + 1), -1.1); s.cdf.push_back(acc); }
  for (double& c : s.cdf) c /= acc;
  return s;
}

std::vector<uint32_t> range_cps(uint32_t base, uint32_t count) {
  std::vector<uint32_t> v;
  for (uint32_t i = 0; i < count; ++i) v.push_back(base + i);
  return v;
}

struct Scripts {
  std::vector<Script> scripts;
  std::vector<double> mix_cdf;  // per-word script choice
};

Scripts make_scripts(const std::string& mode) {
  Scripts S;
  std::vector<uint32_t> latin;
  for (const char* p = "etaoinshrdlcumwfgypbvkjxqz"; *p; ++p) latin.push_back((uint32_t)*p);
  S.scripts.push_back(make_script(latin));
  std::vector<double> w;
  if (mode == "ascii") {
    w = {1.0};
  } else if (mode == "utf8") {
    S.scripts.push_back(make_script(range_cps(0x03B1, 25)));   // Greek small letters
    S.scripts.push_back(make_script(range_cps(0x0430, 32)));   // Cyrillic small letters
    S.scripts.push_back(make_script(range_cps(0x4E00, 2500))); // CJK unified ideographs
    w = {0.70, 0.10, 0.10, 0.10};
  } else if (mode == "mixed") {
    S.scripts.push_back(make_script(range_cps(0x03B1, 25)));   // Greek
    S.scripts.push_back(make_script(range_cps(0x0430, 32)));   // Cyrillic
    S.scripts.push_back(make_script(range_cps(0x4E00, 2500))); // CJK
    S.scripts.push_back(make_script(range_cps(0x0627, 26)));   // Arabic letters
    S.scripts.push_back(make_script(range_cps(0x0905, 40)));   // Devanagari
    S.scripts.push_back(make_script(range_cps(0xAC00, 2000))); // Hangul syllables
    S.scripts.push_back(make_script(range_cps(0x0E01, 46)));   // Thai
    w = {0.40, 0.10, 0.10, 0.10, 0.08, 0.08, 0.07, 0.07};
  } else {
    std::fprintf(stderr, "gen_corpus: unknown script '%s'\n", mode.c_str());
    std::exit(2);
  }
  double acc = 0.0;
  for (double x : w) { acc += x; S.mix_cdf.push_back(acc); }
  for (double& c : S.mix_cdf) c /= acc;
  return S;
}

inline size_t pick(const std::vector<double>& cdf, double u) {
  size_t i = (size_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
  return i < cdf.size() ? i : cdf.size() - 1;
}

inline void put_utf8(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out.push_back((char)cp);
  } else if (cp < 0x800) {
    out.push_back((char)(0xC0 | (cp >> 6)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    out.push_back((char)(0xE0 | (cp >> 12)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  }
}

// Spelling of word type `k` is a pure function of (seed, k).
void spell_word(std::string& out, const Scripts& S, uint64_t seed, uint64_t k) {
  Rng r(splitmix64(seed * 0xD6E8FEB86659FD93ull) ^ splitmix64(k + 0x5851F42D4C957F2Dull));
  const Script& sc = S.scripts[pick(S.mix_cdf, r.uniform())];
  int len = 1;
  while (len < kMaxChars && r.uniform() < 0.8) ++len;
  for (int i = 0; i < len; ++i) put_utf8(out, sc.cps[pick(sc.cdf, r.uniform())]);
}

// The spellings of the most frequent types (Zipf: the first 2^20 types are >= 94% of the words
// even at 100 GB), computed once and copied per occurrence; rarer types are spelled on the fly.
// Same bytes either way.
struct SpellCache {
  std::vector<uint32_t> off;  // kCached + 1
  std::string bytes;
};
constexpr uint64_t kCached = 1u << 20;

SpellCache make_cache(const Scripts& S, uint64_t seed, int threads) {
  SpellCache c;
  std::vector<std::string> part(threads);
  std::vector<std::vector<uint32_t>> lens(threads);
  std::vector<std::thread> pool;
  const uint64_t per = (kCached + threads - 1) / threads;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      const uint64_t k0 = 1 + per * t, k1 = std::min<uint64_t>(kCached + 1, k0 + per);
      for (uint64_t k = k0; k < k1; ++k) {
        const size_t before = part[t].size();
        spell_word(part[t], S, seed, k);
        lens[t].push_back((uint32_t)(part[t].size() - before));
      }
    });
  for (auto& th : pool) th.join();
  c.off.reserve(kCached + 1);
  c.off.push_back(0);
  for (int t = 0; t < threads; ++t) {
    for (uint32_t l : lens[t]) c.off.push_back(c.off.back() + l);
    c.bytes += part[t];
  }
  return c;
}

inline void emit_word(std::string& out, const Scripts& S, const SpellCache& c, uint64_t seed, uint64_t k) {
  if (k <= kCached) out.append(c.bytes, c.off[k - 1], c.off[k] - c.off[k - 1]);
  else spell_word(out, S, seed, k);
}

void gen_block(std::string& out, const Scripts& S, const SpellCache& c, uint64_t seed, uint64_t block) {
  out.clear();
  const double n_end = (double)(block + 1) * kLinesPerBlock * kWordsPerLine;
  uint64_t universe = (uint64_t)std::ceil(30.0 * std::pow(n_end, 0.55));
  if (universe < 64) universe = 64;
  Zipf z(universe, 1.1);
  Rng r(splitmix64(seed) ^ splitmix64(block * 0x9E3779B97F4A7C15ull + 1));
  for (int l = 0; l < kLinesPerBlock; ++l) {
    for (int w = 0; w < kWordsPerLine; ++w) {
      emit_word(out, S, c, seed, z.sample(r));
      out.push_back(w + 1 < kWordsPerLine ? ' ' : '\n');
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  uint64_t bytes = 0, seed = 1;
  std::string script = "ascii", out_path;
  int threads = (int)std::thread::hardware_concurrency();
  if (const char* e = std::getenv("OMP_NUM_THREADS")) threads = std::max(1, std::atoi(e));
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string k = argv[i], v = argv[i + 1];
    if (k == "--bytes") bytes = std::strtoull(v.c_str(), nullptr, 10);
    else if (k == "--seed") seed = std::strtoull(v.c_str(), nullptr, 10);
    else if (k == "--script") script = v;
    else if (k == "--out") out_path = v;
    else if (k == "--threads") threads = std::max(1, std::atoi(v.c_str()));
    else { std::fprintf(stderr, "gen_corpus: unknown flag %s\n", k.c_str()); return 2; }
  }
  if (!bytes || out_path.empty()) {
    std::fprintf(stderr, "usage: gen_corpus --bytes N --seed S --script ascii|utf8|mixed --out PATH [--threads T]\n");
    return 2;
  }
  threads = std::min(threads, 64);
  const Scripts S = make_scripts(script);
  const SpellCache cache = make_cache(S, seed, threads);
  FILE* f = std::fopen(out_path.c_str(), "wb");
  if (!f) { std::perror("gen_corpus: fopen"); return 1; }
  // rounds of `threads` blocks; round r is written by a writer thread while round r + 1 is made
  std::vector<std::string> bufs[2] = {std::vector<std::string>(threads), std::vector<std::string>(threads)};
  uint64_t written = 0, block = 0;
  bool write_err = false;
  std::thread writer;
  int cur = 0;
  while (written < bytes) {
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) pool.emplace_back([&, t] { gen_block(bufs[cur][t], S, cache, seed, block + t); });
    for (auto& th : pool) th.join();
    if (writer.joinable()) writer.join();
    if (write_err) { std::perror("gen_corpus: fwrite"); return 1; }
    // what this round contributes (the last byte of the file is '\n')
    uint64_t take_total = 0;
    for (int t = 0; t < threads; ++t) {
      std::string& b = bufs[cur][t];
      const uint64_t take = std::min<uint64_t>(b.size(), bytes - written - take_total);
      if (take && written + take_total + take == bytes) b[take - 1] = '\n';
      b.resize(take);
      take_total += take;
    }
    writer = std::thread([&, c = cur] {
      for (std::string& b : bufs[c])
        if (!b.empty() && std::fwrite(b.data(), 1, b.size(), f) != b.size()) write_err = true;
    });
    written += take_total;
    block += threads;
    cur ^= 1;
  }
  if (writer.joinable()) writer.join();
  if (write_err) { std::perror("gen_corpus: fwrite"); return 1; }
  if (std::fclose(f) != 0) { std::perror("gen_corpus: fclose"); return 1; }
  return 0;
}
