// C ABI of the BPE encoder (include/shredword_encode.h): reads the trainer's
// .model / .vocab files (written by reference bpe.cpp:388-432), validates the merge list, builds
// the merge-rank table and the byte map, and hands the text to the gfx950 kernels
// (encode_device.hip).  There is no host encoder: without a device the calls fail.
#include "shredword_encode.h"

#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "encoder.h"

namespace shred {

std::vector<uint64_t> enc_build_table(const std::vector<int32_t>& first, const std::vector<int32_t>& second) {
  size_t cap = 1024;
  while (cap < 2 * first.size()) cap <<= 1;
  std::vector<uint64_t> tab(cap, kEncEmpty);
  const uint64_t mask = cap - 1;
  for (size_t m = 0; m < first.size(); ++m) {
    const uint64_t key = enc_key(first[m], second[m]);
    for (uint64_t i = enc_slot(key) & mask;; i = (i + 1) & mask) {
      if (tab[i] == kEncEmpty) {
        tab[i] = key << 20 | (uint64_t)m;
        break;
      }
      if ((tab[i] >> 20) == key) break;  // a repeated pair: the lowest rank already holds it
    }
  }
  return tab;
}

}  // namespace shred

struct ShredEncoder {
  std::vector<int32_t> first, second;
  int32_t byte_map[256];
  std::vector<std::string> tokens;  // bytes of every id (256 + merges)
  std::unique_ptr<shred::EncodeDevice> dev;
};

namespace {

bool read_file(const char* path, std::string* out) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  char buf[1 << 16];
  size_t r;
  out->clear();
  while ((r = std::fread(buf, 1, sizeof buf, f)) > 0) out->append(buf, r);
  std::fclose(f);
  return true;
}

ShredEncoder* make(std::vector<int32_t> first, std::vector<int32_t> second, const int32_t* byte_map, int device) {
  const size_t M = first.size();
  if (M + 256 > (size_t)shred::kEncIdLimit) {
    std::fprintf(stderr, "[ERROR]\t encoder: %zu merges exceed the id limit 2^20\n", M);
    return nullptr;
  }
  std::unique_ptr<ShredEncoder> e(new ShredEncoder());
  for (int b = 0; b < 256; ++b) e->byte_map[b] = byte_map ? byte_map[b] : b;
  e->tokens.resize(256 + M);
  for (int b = 0; b < 256; ++b) e->tokens[b] = std::string(1, (char)b);
  for (size_t m = 0; m < M; ++m) e->tokens[256 + m] = e->tokens[first[m]] + e->tokens[second[m]];
  std::string why;
  e->dev.reset(shred::EncodeDevice::create(device, shred::enc_build_table(first, second), e->byte_map, &why));
  if (!e->dev) {
    std::fprintf(stderr, "[ERROR]\t encoder: %s\n", why.c_str());
    return nullptr;
  }
  e->first = std::move(first);
  e->second = std::move(second);
  return e.release();
}

bool split_merges(const int32_t* triples, size_t M, std::vector<int32_t>* first, std::vector<int32_t>* second) {
  first->resize(M);
  second->resize(M);
  for (size_t m = 0; m < M; ++m) {
    const int32_t a = triples[3 * m], b = triples[3 * m + 1], id = triples[3 * m + 2];
    if (id != (int32_t)(256 + m) || a < 0 || b < 0 || a >= id || b >= id) {
      std::fprintf(stderr, "[ERROR]\t encoder: merge %zu (%d, %d -> %d) is not a trainer merge\n", m, a, b, id);
      return false;
    }
    (*first)[m] = a;
    (*second)[m] = b;
  }
  return true;
}

// Frequency column of a .vocab file: record i is "<token i without NUL bytes> <freq>\n" (the
// reference prints C strings, bpe.cpp:394-417).  False when the file does not match the tokens.
bool vocab_freqs(const std::string& v, const std::vector<std::string>& tokens, std::vector<uint64_t>* freq) {
  size_t pos = 0;
  freq->assign(tokens.size(), 0);
  for (size_t i = 0; i < tokens.size(); ++i) {
    for (char c : tokens[i]) {
      if (c == 0) continue;
      if (pos >= v.size() || v[pos] != c) return false;
      ++pos;
    }
    if (pos >= v.size() || v[pos] != ' ') return false;
    ++pos;
    uint64_t f = 0;
    size_t digits = 0;
    while (pos < v.size() && v[pos] >= '0' && v[pos] <= '9') f = f * 10 + (uint64_t)(v[pos++] - '0'), ++digits;
    if (!digits || pos >= v.size() || v[pos] != '\n') return false;
    ++pos;
    (*freq)[i] = f;
  }
  return pos == v.size();
}

}  // namespace

extern "C" {

ShredEncoder* shred_encoder_create(const int32_t* merges, size_t num_merges, const int32_t* byte_map, int device) {
  if (!merges && num_merges) return nullptr;
  std::vector<int32_t> first, second;
  if (!split_merges(merges, num_merges, &first, &second)) return nullptr;
  return make(std::move(first), std::move(second), byte_map, device);
}

ShredEncoder* shred_encoder_load(const char* model_path, const char* vocab_path, int32_t unk_id, int device) {
  if (!model_path) return nullptr;
  std::string model;
  if (!read_file(model_path, &model)) {
    std::fprintf(stderr, "[ERROR]\t encoder: couldn't open %s\n", model_path);
    return nullptr;
  }
  if (model.size() % 12) {
    std::fprintf(stderr, "[ERROR]\t encoder: %s is not a sequence of int32 triples\n", model_path);
    return nullptr;
  }
  const size_t M = model.size() / 12;
  std::vector<int32_t> triples(3 * M);
  if (M) std::memcpy(triples.data(), model.data(), model.size());
  std::vector<int32_t> first, second;
  if (!split_merges(triples.data(), M, &first, &second)) return nullptr;
  int32_t map[256];
  for (int b = 0; b < 256; ++b) map[b] = b;
  if (vocab_path) {
    std::string vocab;
    if (!read_file(vocab_path, &vocab)) {
      std::fprintf(stderr, "[ERROR]\t encoder: couldn't open %s\n", vocab_path);
      return nullptr;
    }
    std::vector<std::string> tokens(256 + M);
    for (int b = 0; b < 256; ++b) tokens[b] = std::string(1, (char)b);
    for (size_t m = 0; m < M; ++m) tokens[256 + m] = tokens[first[m]] + tokens[second[m]];
    std::vector<uint64_t> freq;
    if (!vocab_freqs(vocab, tokens, &freq)) {
      std::fprintf(stderr, "[ERROR]\t encoder: %s does not match the merges of %s\n", vocab_path, model_path);
      return nullptr;
    }
    // a byte the coverage rule dropped never has a symbol of its own and never merges
    bool used[256] = {false};
    for (size_t m = 0; m < M; ++m) {
      if (first[m] < 256) used[first[m]] = true;
      if (second[m] < 256) used[second[m]] = true;
    }
    for (int b = 0; b < 256; ++b)
      if (freq[b] == 0 && !used[b]) map[b] = unk_id;
  }
  return make(std::move(first), std::move(second), map, device);
}

void shred_encoder_destroy(ShredEncoder* enc) { delete enc; }

int shred_encoder_info(const ShredEncoder* enc, size_t* num_merges, int32_t* byte_map) {
  if (!enc) return -1;
  if (num_merges) *num_merges = enc->first.size();
  if (byte_map) std::memcpy(byte_map, enc->byte_map, sizeof enc->byte_map);
  return 0;
}

int64_t shred_encode(ShredEncoder* enc, const uint8_t* text, size_t n, int32_t* out, size_t cap) {
  if (!enc || (n && (!text || !out))) return -1;
  return enc->dev->encode_host(text, n, out, cap);
}

int64_t shred_encode_device(ShredEncoder* enc, const void* text, size_t n, void* out, size_t cap, void* stream,
                            double* kernel_ms) {
  if (!enc || (n && (!text || !out))) return -1;
  return enc->dev->encode((const uint8_t*)text, n, (int32_t*)out, cap, stream, kernel_ms);
}

int64_t shred_decode(const ShredEncoder* enc, const int32_t* ids, size_t n, uint8_t* out, size_t cap) {
  if (!enc || (n && !ids)) return -1;
  size_t need = 0;
  for (size_t i = 0; i < n; ++i) {
    if (ids[i] < 0 || (size_t)ids[i] >= enc->tokens.size()) return -1;
    const std::string& t = enc->tokens[ids[i]];
    if (out && need + t.size() <= cap) std::memcpy(out + need, t.data(), t.size());
    need += t.size();
  }
  return (int64_t)need;
}

}  // extern "C"
