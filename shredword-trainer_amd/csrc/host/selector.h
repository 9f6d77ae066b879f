// Exact merge selection for the BPE path: the host half of the merge loop.
//
// The device finds every occurrence of the merged pair and reduces its neighbour-pair deltas;
// this class turns those deltas into the reference's exact pair-info updates and heap pushes,
// and replays the reference heap to pick the next merge.  Merge order is decided by ties in the
// reference's binary heap (SURVEY.md §0 finding 2), so bit-exact output needs this replay:
//
//  * pair info      Info{freq, version} per pair (reference hash.h:31-45, bimap_get hash.cpp:104-130)
//  * heap           push sifts up while parent < child; pop sifts down left-first, right only
//                   if strictly greater (reference heap.cpp:53-114)
//  * select         bpe_merge_batch's pop loop (bpe.cpp:244-258); the O(S) recompute_freq
//                   (bpe.cpp:52-65) is replaced by its provable value: 0 for keys holding unk,
//                   info.freq otherwise (deltas keep non-unk counts exact, SURVEY.md §0 finding 3).
//                   That holds while the pair info IS the corpus's count (exact()): after a bpe_init,
//                   or a count on the fresh pair map of a load.  Call sequences that break it (a
//                   count on a counted map doubles it, bpe.cpp:207-211; merge_batch after a load
//                   without a count pops the old corpus's heap over a fresh map, :176-183) take the
//                   rescan's value from a truth table: one device recount, then the merges' exact
//                   deltas (set_truth / truth_live).
//  * apply          the FreqChangeMap semantics of bpe.cpp:265-313: deltas keyed by
//                   ((i64)first << 32) | (i64)second (sign-extension folds every (x, negative) key
//                   to (-1, negative)), applied bucket (key % 1024) ascending and, inside a bucket,
//                   in reverse order of first touch, clamped at 0, net-zero entries included.
#pragma once

#include <sys/mman.h>

#include <cstddef>
#include <cstdint>
#include <new>
#include <unordered_map>
#include <vector>

namespace shred {

// Allocator for the selector's big random-access arrays (pair table, heap): 2 MiB-aligned
// anonymous mappings marked MADV_HUGEPAGE, so a lookup or a heap level costs a cache miss and
// not also a page walk (at C3 the pair table is ~400 MB and the heap ~70 MB).  Small requests
// use operator new.
template <class T>
struct HugeAlloc {
  using value_type = T;
  static constexpr size_t kHuge = size_t(1) << 21;
  HugeAlloc() = default;
  template <class U>
  HugeAlloc(const HugeAlloc<U>&) {}
  T* allocate(size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes < kHuge) return static_cast<T*>(::operator new(bytes));
    const size_t len = (bytes + kHuge - 1) & ~(kHuge - 1);
    char* p = static_cast<char*>(mmap(nullptr, len + kHuge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
    if (p == MAP_FAILED) throw std::bad_alloc();
    char* a = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(p) + kHuge - 1) & ~(uintptr_t)(kHuge - 1));
    if (a > p) munmap(p, a - p);
    if (a + len < p + len + kHuge) munmap(a + len, (p + len + kHuge) - (a + len));
    madvise(a, len, MADV_HUGEPAGE);
    return reinterpret_cast<T*>(a);
  }
  void deallocate(T* ptr, size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes < kHuge) {
      ::operator delete(ptr);
      return;
    }
    munmap(ptr, (bytes + kHuge - 1) & ~(kHuge - 1));
  }
  template <class U>
  bool operator==(const HugeAlloc<U>&) const { return true; }
  template <class U>
  bool operator!=(const HugeAlloc<U>&) const { return false; }
};
template <class T>
using HugeVec = std::vector<T, HugeAlloc<T>>;

// One device delta record: key = slot * 4 + category (see DeltaCategory); the neighbour id is
// slot - 1, slot 0 standing for unk_id when unk_id lies outside [0, slot capacity).
struct DeltaRecord {
  uint32_t key;
  uint32_t pad;
  uint64_t sum;  // Σ word weight over the occurrences (magnitude; sign given by the category)
  uint64_t ft;   // first touch: (word rank << 32) | (position in word << 2) | category
};
static_assert(sizeof(DeltaRecord) == 24, "DeltaRecord layout is shared with the device");

enum DeltaCategory : uint32_t {
  kOldLeft = 0,   // (p, a)  -= w   (bpe.cpp:276-279)
  kNewLeft = 1,   // (p, X)  += w
  kOldRight = 2,  // (b, n)  -= w   (bpe.cpp:283-289)
  kNewRight = 3,  // (X, n)  += w
};

struct PairCount {
  int32_t a, b;
  uint64_t count;
  uint64_t ft;  // first touch (word rank << 32) | position: the reference bimap creation order
};

// tiebreak=device (opt-in, not the reference's order): a merge the device selected itself.
struct SelectedMerge {
  int32_t a, b;
  uint64_t freq;
};

class Selector {
 public:
  // One merge's records combined per pair and put in the reference's application order: the part
  // of apply() that reads nothing of the selector's state, so another thread can make it while the
  // selector selects (Engine's apply helper).
  struct Change { uint64_t hk; int64_t delta; uint64_t ft; };
  struct Prepared {
    int32_t a = 0, b = 0, X = 0;
    size_t records = 0;
    std::vector<Change> changes, staged, ordered;
    std::vector<uint32_t> index;
    uint64_t cyc_combine = 0, cyc_order = 0;
  };
  // K4 done on the device (word_loop.hip finalize_changes): the merge's changes already combined
  // per pair key and in the reference's application order (bucket ascending, first touch
  // descending); the next apply_finish walks them as they are.
  void apply_changes(int32_t a, int32_t b, int32_t X, const Change* c, size_t n);
  // Thread-safe against every other member: reads only unk_ (fixed during a train()).
  // prefetch_base / prefetch_mask: a snapshot of the pair table to prefetch the changed pairs'
  // lines from (nullptr: none).
  void prepare(int32_t a, int32_t b, int32_t X, const DeltaRecord* recs, size_t n, Prepared* p,
               const void* prefetch_base, uint64_t prefetch_mask) const;
  // The table snapshot for prepare() on another thread.
  const void* table_base() const { return table_.data(); }
  uint64_t table_mask() const { return mask_; }
  // A merge prepared elsewhere becomes the current one (as after apply_combine); p gets the old
  // buffers back for reuse.
  void adopt(Prepared* p);

  // bpe_init's fresh pair map and heap (bpe.cpp:103-106).
  void reset(int32_t unk_id, uint64_t min_pair_freq);
  // bpe_load_corpus: a fresh pair map (bpe.cpp:183); the heap and its entries stay.
  void reset_info();

  // bpe_count_bigrams (bpe.cpp:187-230): adds counts (new pairs created in first-touch order),
  // then pushes every pair with freq >= min in (FNV bucket & 4095, creation order).
  void add_counts(std::vector<PairCount> pairs);

  // bpe_merge_batch's pop loop: true with the pair to merge and its freq; false if the heap
  // ran empty.
  bool select(int32_t* a, int32_t* b, uint64_t* freq);

  // Applies one merge's device deltas and finalises the merged key (bpe.cpp:297-318).
  void apply(int32_t a, int32_t b, int32_t X, const DeltaRecord* recs, size_t n);
  // apply() in two steps: the records combined into per-pair changes, then the changes applied
  // in the reference's order.  Between them predict_after() can see the changes.
  void apply_combine(int32_t a, int32_t b, int32_t X, const DeltaRecord* recs, size_t n);
  void apply_finish(int32_t a, int32_t b, int32_t X);
  // Between the two steps: the most frequent new pair holding X (its count is exact: the pair
  // did not exist before this merge) if its count is above `above` -- a better guess of the next
  // merge than one made before (a, b)'s records were known.
  bool predict_after(int32_t X, uint64_t above, int32_t* pa, int32_t* pb, uint64_t* pf) const;

  // Guess of the merge after (a, b), made before (a, b)'s deltas are known: the best valid heap
  // entry among the first `window` heap slots that shares no token with (a, b).  Used only to
  // run the next merge speculatively; the exact replay decides.
  bool predict_next(int32_t a, int32_t b, size_t window, int32_t* pa, int32_t* pb) const;
  // The same with every token in used[0, n_used) avoided (deeper speculation: the guess after
  // the guesses already in flight).
  bool predict_avoid(const int32_t* used, size_t n_used, size_t window, int32_t* pa, int32_t* pb) const;
  // Up to k further merges guessed from the heap after (a, b): the best valid entries that
  // share no token with (a, b) or with each other, by frequency.  out: k (a, b) pairs.
  size_t predict_chain(int32_t a, int32_t b, size_t window, size_t k, int32_t* out) const;

  // predict_avoid refines its guess by replaying the coming select() on an overlay of the heap
  // (simulate_select); off: the slot-order guess alone.
  void set_simulate_pops(bool on) { simulate_pops_ = on; }

  // True while every pair's info equals its count in the corpus (recompute_freq is then
  // info.freq).  Otherwise select() needs the truth table.
  bool exact() const { return exact_; }
  // Debug check of exact(): the number of pairs, unk pairs aside, whose info differs
  // from `fresh` (a fresh K1 of the corpus), counting pairs present on one side only.
  size_t exact_mismatches(const std::vector<PairCount>& fresh) const;
  bool truth_live() const { return truth_live_; }
  // The corpus's pair counts now (a fresh K1): recompute_freq's values until the corpus changes;
  // each applied merge then updates them by its exact deltas.
  void set_truth(const std::vector<PairCount>& pairs);

  size_t heap_size() const { return heap_.empty() ? 0 : heap_.size() - 1; }
  bool heap_empty() const { return heap_.size() <= 1; }
  uint64_t heap_top_freq() const { return heap_empty() ? 0 : node_freq(heap_[1]); }
  size_t num_pairs() const { return count_; }
  // freq/version of a pair (0/0 when absent); for tests.
  bool lookup(int32_t a, int32_t b, uint64_t* freq, uint32_t* version) const;
  int32_t unk_id() const { return unk_; }
  struct Counters {
    uint64_t pops = 0, stale = 0, pushes = 0, records = 0, changes = 0;
    uint64_t cyc_combine = 0, cyc_order = 0, cyc_walk = 0, cyc_push = 0;  // TSC cycles inside apply()
  };
  const Counters& counters() const { return ctr_; }
  size_t last_records() const { return own_.records; }  // the current merge's delta records

 private:
  // One flat open-addressing table: a lookup touches one cache line.  kEmptyKey is the packed
  // pair (INT32_MIN, INT32_MIN), which no token pair can be (ids are >= -2^30).
  // 16 bytes: four to a cache line.  freq (40 bits) << 24 | version (24 bits); the creation
  // sequence number the heap build orders by lives beside, in seq_.
  struct Info {
    uint64_t key;
    uint64_t fv;
    uint64_t freq() const { return fv >> 24; }
    uint32_t version() const { return (uint32_t)(fv & 0xFFFFFFu); }
    void set_freq(uint64_t f) {
      if (f >> 40) info_overflow();
      fv = f << 24 | (fv & 0xFFFFFFu);
    }
    void set_version(uint32_t v) { fv = (fv & ~0xFFFFFFull) | (v & 0xFFFFFFu); }
    void bump_version() {
      if ((fv & 0xFFFFFFu) == 0xFFFFFFu) info_overflow();
      ++fv;
    }
  };
  [[noreturn]] static void info_overflow();
  struct HeapEnt { int32_t a, b; uint64_t freq; uint32_t version; };
  // A heap node in 16 bytes: frequency (40 bits) << 24 | version (24 bits), then the pair.
  struct HeapNode { uint64_t fv; int32_t a, b; };
  static uint64_t node_freq(const HeapNode& n) { return n.fv >> 24; }
  static uint32_t node_version(const HeapNode& n) { return (uint32_t)(n.fv & 0xFFFFFFu); }
  static constexpr uint64_t kEmptyKey = 0x8000000080000000ull;

  Info& get(int32_t a, int32_t b);  // get-or-create (bimap_get)
  const Info* find(uint64_t key) const;
  void push(int32_t a, int32_t b, uint64_t freq, uint32_t version);
  HeapEnt pop();
  void grow();

  int32_t unk_ = 0;
  uint64_t min_freq_ = 2000;
  HugeVec<Info> table_;
  // Creation order (bimap_get order) of every pair since the last fresh map: the heap build of a
  // count pushes in (bucket, creation) order, and a count may come after merges created pairs.
  // An append-only log (a sequential store per new pair, not a random one).
  std::vector<uint64_t> created_;
  size_t count_ = 0;
  bool exact_ = true;
  bool truth_live_ = false;
  std::unordered_map<uint64_t, uint64_t> truth_;  // pair -> its count in the corpus (non-exact state)
  uint64_t recount(int32_t a, int32_t b) const;
  uint64_t mask_ = 0;
  // The reference's binary heap (heap.cpp), logical slot k stored at heap_[k + 1]: with 16-byte
  // nodes on a 2 MiB-aligned array, the two children of a slot share one 32-byte half line and
  // its four grandchildren one 64-byte line, so a sift level touches one cache line (frequency
  // and payload together).  heap_[0] is padding.
  HugeVec<HeapNode> heap_;
  Prepared own_;  // the current merge's changes (apply_combine / adopt -> apply_finish)
  std::vector<HeapNode> pushes_;  // apply: the pushes of one merge, in order
  bool simulate_select(const int32_t* used, size_t n_used, uint64_t floor, int32_t* pa, int32_t* pb) const;
  bool simulate_pops_ = true;
  // simulate_select's overlay: heap slot -> node, valid where the stamp equals the generation
  mutable std::vector<uint32_t> ov_stamp_;
  mutable std::vector<size_t> ov_pos_;
  mutable std::vector<HeapNode> ov_node_;
  mutable uint32_t ov_gen_ = 0;
  Counters ctr_;
};

}  // namespace shred
