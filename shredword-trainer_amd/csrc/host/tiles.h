// The tiled token stream that lives in HBM (see DESIGN.md "Data layout").
//
// Entries (distinct words in the "types" layout, word occurrences in corpus order in the
// "stream" layout) are packed whole into tiles of at most kTileTokens tokens; a word longer than
// that gets a tile of its own.  Each entry is written as an in-band header INT32_MIN + rank
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
  size_t num_tiles() const { return len.size(); }
};

// Number of entries of the layout (distinct words or occurrences).
size_t layout_entries(const WordTable& wt, Layout layout);
// This rank's contiguous share of the entries, balanced by token count.
void shard_range(const WordTable& wt, Layout layout, int rank, int world, size_t* begin, size_t* end);
// Packs entries [begin, end) into tiles.
void pack_tiles(const WordTable& wt, Layout layout, size_t begin, size_t end, TiledStream* out);

}  // namespace shred
