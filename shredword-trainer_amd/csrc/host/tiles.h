// The tiled token stream that lives in HBM (see DESIGN.md "Data layout").
//
// Entries (distinct words in the "types" layout, word occurrences in corpus order in the
// "stream" layout) are packed whole into tiles of at most kTileTokens tokens; a word longer than
// that gets a tile of its own (the stream layout packs the first occurrence of every type
// first, see pack_tiles).  Each entry is written as an in-band header INT32_MIN + rank
// followed by its symbol ids.  Tiles start 16-byte aligned.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include "corpus.h"

namespace shred {

enum class Layout { kTypes = 0, kStream = 1 };

constexpr uint32_t kTileTokens = 1024;  // one wave64 chunk (64 lanes x 16 tokens)

struct TiledStream {
  std::vector<int32_t> tok;    // elems + 4 tokens, padding = INT32_MIN
  std::vector<uint64_t> off;   // per tile: element offset
  std::vector<uint32_t> len;   // per tile: live length (headers included)
  uint64_t elems = 0;
  uint64_t live = 0;           // Σ len
  size_t entries = 0;
  size_t ft_tiles = 0;         // tiles [0, ft_tiles) hold one occurrence of every type (all tiles in
                               // the types layout); K1 takes first touch from them alone
  size_t num_tiles() const { return len.size(); }
};

// Number of entries of the layout (distinct words or occurrences).
size_t layout_entries(const WordTable& wt, Layout layout);
// This rank's contiguous share of the entries, balanced by token count.
void shard_range(const WordTable& wt, Layout layout, int rank, int world, size_t* begin, size_t* end);
// Packs entries [begin, end) into tiles.
void pack_tiles(const WordTable& wt, Layout layout, size_t begin, size_t end, TiledStream* out);

}  // namespace shred

namespace shred {

// Tile skipping: for every token id, a superset of the tiles that hold it.
// A merge (a, b) only has to visit tiles(a) ∩ tiles(b); the merge reports the tiles where it
// created X, which become tiles(X).  A merge never creates an adjacency between two tokens
// that both existed before it, so for pairs of two base ids (< 256) the exact tile list of
// the initial stream stays a superset for the whole run and replaces the intersection.  Sets
// with few tiles are sorted lists, frequent ones bitmaps.  Supersets stay correct, so nothing
// is removed after a merge.
class TileIndex {
 public:
  void build(const TiledStream& ts);
  void reset();  // back to the state after build()
  // Candidate tiles of (a, b) in ascending order; false = visiting every tile is cheaper.
  bool candidates(int32_t a, int32_t b, std::vector<uint32_t>* out) const;
  // The owners of (a, b)'s candidate tiles, where owner w holds tiles [first[w], first[w+1]):
  // ascending workgroup ids in *out.  Computed on tile bitmaps without listing the tiles.
  void owners(int32_t a, int32_t b, const std::vector<uint32_t>& first, std::vector<uint32_t>* out) const;
  void set_tiles(int32_t id, const uint32_t* tiles, size_t n);
  // The same from a bitmap over the tiles ((ntiles + 31) / 32 words, bit t = tile t) of n bits.
  void set_tiles_bits(int32_t id, const uint32_t* words, size_t n);
  void set_all(int32_t id);  // id may be in any tile
  size_t num_tiles() const { return ntiles_; }

 private:
  struct Set {
    std::vector<uint32_t> list;  // sorted, when sparse
    std::vector<uint64_t> bits;  // when dense
    size_t size = 0;
  };
  void make(Set* s, std::vector<uint32_t>&& sorted) const;
  const Set* get(int32_t id) const { return (id >= 0 && (size_t)id < ids_.size()) ? &ids_[id] : nullptr; }

  bool intersect(const Set* sa, const Set* sb, std::vector<uint32_t>* out) const;

  void to_bits(const Set* s, std::vector<uint64_t>* bits) const;
  uint32_t ntiles_ = 0;
  std::vector<Set> ids_, ids0_;
  mutable std::vector<uint64_t> ba_, bb_;  // scratch bitmaps of owners()
  std::vector<Set> base_pairs_;  // [a * 256 + b] for a, b < 256 (immutable after build)
};

}  // namespace shred
