/* encode_oracle.c — TEST INFRASTRUCTURE ONLY (the checker of the GPU encoder).
 * Never linked into the product; only tests/ and bench.py's cpu_baseline leg call it.
 *
 * Clean-room restatement of the encoding include/shredword_encode.h defines: the reference
 * trainer's merge application (shredword/csrc/bpe/bpe.cpp:265-296) replayed literally on every
 * word of the text, merge 0 first.  Within one merge the scan re-tests the merged symbol and moves
 * on (bpe.cpp:268-272, 292-295), i.e. left to right without overlap.  Words are the runs of bytes
 * outside "\t\r\n " (the strtok split, bpe.cpp:143-153); byte b becomes byte_map[b].  Distinct
 * words are encoded once (a cache keyed by the word's bytes) so 2-10 MB corpora take seconds.
 *
 * Pinned by the reference's own outputs: on a golden corpus (tests/golden) the counts of the ids
 * this produces equal the frequency column of the reference's .vocab (tests/test_encode_oracle.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ENC_MAX_WORD 1024

static int is_delim(unsigned char c) { return c == '\t' || c == '\r' || c == '\n' || c == ' '; }

typedef struct {
  size_t text_off;  /* first occurrence in the text (word bytes) */
  uint32_t len;
  size_t ids_off;   /* into the id pool */
  uint32_t nids;
  int used;
} Slot;

static uint64_t fnv(const unsigned char* p, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

/* Replays merges[0..M) on syms[0..n); returns the final length. */
static size_t replay(const int32_t* merges, size_t M, int32_t* syms, size_t n) {
  for (size_t m = 0; m < M && n > 1; ++m) {
    const int32_t a = merges[3 * m], b = merges[3 * m + 1], x = (int32_t)(256 + m);
    size_t i = 0;
    while (i + 1 < n) {
      if (syms[i] != a || syms[i + 1] != b) { ++i; continue; }
      syms[i] = x;  /* the symbol stays and is re-tested; x never equals a */
      memmove(syms + i + 1, syms + i + 2, (n - i - 2) * sizeof(int32_t));
      --n;
    }
  }
  return n;
}

/* Returns the number of ids, -2 when cap is too small, -3 for a word longer than ENC_MAX_WORD,
 * -1 on allocation failure.  byte_map NULL = identity. */
int64_t or_encode(const int32_t* merges, size_t M, const int32_t* byte_map, const unsigned char* text, size_t n,
                  int32_t* out, size_t cap) {
  size_t nslots = 1 << 16;
  Slot* slots = calloc(nslots, sizeof(Slot));
  size_t used = 0, pool_cap = 1 << 20, pool_n = 0;
  int32_t* pool = malloc(pool_cap * sizeof(int32_t));
  int32_t syms[ENC_MAX_WORD];
  int64_t total = 0;
  if (!slots || !pool) { free(slots); free(pool); return -1; }
  size_t i = 0;
  while (i < n) {
    while (i < n && is_delim(text[i])) ++i;
    if (i >= n) break;
    size_t s = i;
    while (i < n && !is_delim(text[i])) ++i;
    size_t L = i - s;
    if (L > ENC_MAX_WORD) { free(slots); free(pool); return -3; }
    if (2 * (used + 1) > nslots) {  /* grow the cache */
      size_t ncap = nslots * 2;
      Slot* ns = calloc(ncap, sizeof(Slot));
      if (!ns) { free(slots); free(pool); return -1; }
      for (size_t k = 0; k < nslots; ++k) {
        if (!slots[k].used) continue;
        size_t h = fnv(text + slots[k].text_off, slots[k].len) & (ncap - 1);
        while (ns[h].used) h = (h + 1) & (ncap - 1);
        ns[h] = slots[k];
      }
      free(slots);
      slots = ns;
      nslots = ncap;
    }
    size_t h = fnv(text + s, L) & (nslots - 1);
    while (slots[h].used && !(slots[h].len == L && !memcmp(text + slots[h].text_off, text + s, L)))
      h = (h + 1) & (nslots - 1);
    if (!slots[h].used) {
      for (size_t k = 0; k < L; ++k) syms[k] = byte_map ? byte_map[text[s + k]] : (int32_t)text[s + k];
      size_t m = replay(merges, M, syms, L);
      if (pool_n + m > pool_cap) {
        while (pool_n + m > pool_cap) pool_cap *= 2;
        int32_t* np = realloc(pool, pool_cap * sizeof(int32_t));
        if (!np) { free(slots); free(pool); return -1; }
        pool = np;
      }
      memcpy(pool + pool_n, syms, m * sizeof(int32_t));
      slots[h] = (Slot){s, (uint32_t)L, pool_n, (uint32_t)m, 1};
      pool_n += m;
      ++used;
    }
    if ((size_t)total + slots[h].nids > cap) { free(slots); free(pool); return -2; }
    memcpy(out + total, pool + slots[h].ids_off, slots[h].nids * sizeof(int32_t));
    total += slots[h].nids;
  }
  free(slots);
  free(pool);
  return total;
}
