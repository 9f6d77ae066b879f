// Test-only: the CPU harness (product host sources + kernel emulation) as one executable built
// with AddressSanitizer and UBSan (make -C tests/native asan), so the host logic runs under the
// sanitizers without preloading anything into Python.  tests/test_host_sanitizers.py runs it on
// golden corpora and compares the files with the reference's.
//   hh_asan CORPUS VOCAB UNK COVERAGE MIN_PAIR_FREQ LAYOUT(0 types|1 stream) MODEL VOCABF TRACE [CHAIN]
#include <cstdint>
#include <cstdio>
#include <cstdlib>

extern "C" {
void* hh_open(const char* path, uint64_t vocab, int32_t unk, float cov, uint64_t mpf, int layout, int rank, int world);
void hh_close(void* p);
int hh_train(void* p, const char* trace_path);
void hh_save(void* p, const char* model, const char* vocab, int write);
void hh_set_chain(void* p, int n);
}

int main(int argc, char** argv) {
  if (argc < 10) {
    std::fprintf(stderr, "usage: hh_asan CORPUS VOCAB UNK COVERAGE MPF LAYOUT MODEL VOCABF TRACE [CHAIN]\n");
    return 2;
  }
  void* h = hh_open(argv[1], std::strtoull(argv[2], nullptr, 10), (int32_t)std::atoi(argv[3]),
                    std::strtof(argv[4], nullptr), std::strtoull(argv[5], nullptr, 10), std::atoi(argv[6]), 0, 1);
  if (!h) {
    std::fprintf(stderr, "cannot open %s\n", argv[1]);
    return 1;
  }
  if (argc > 10) hh_set_chain(h, std::atoi(argv[10]));
  const int merges = hh_train(h, argv[9]);
  hh_save(h, argv[7], argv[8], 1);
  hh_close(h);
  std::printf("%d\n", merges);
  return 0;
}
