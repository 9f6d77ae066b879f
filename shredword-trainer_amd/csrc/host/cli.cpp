// `trainer key=value ...` — the reference CLI surface (shredword/csrc/trainer.cpp:30-118, 188-213)
// for the BPE model type, on the MI355X trainer.
//
//   trainer input=corpus.txt model_type=bpe output_model=bpe.model output_vocab=bpe.vocab
//           [vocab_size=32000] [character_coverage=0.9995] [min_pair_freq=2000]
//
// Same keys, defaults and exit codes as the reference: tokens without '=' and unknown keys are
// ignored, missing required keys or a bad model_type print the usage and exit 1, a failed load or
// train exits 255.  unk_id is fixed at -1 as in the reference (trainer.cpp:47); unlike the
// reference this build does not write freq[-1] out of bounds, so it exits 0 after saving.
// model_type=unigram is recognised but not supported by this build (exit 1).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../../include/shredword_bpe.h"

namespace {

void usage(const char* prog) {
  std::printf("Usage: %s <args>\n\n", prog);
  std::printf("Arguments (use: key=value format):\n");
  std::printf("  input=<path>              Input corpus file\n");
  std::printf("  model_type=<bpe|unigram>  Model type\n");
  std::printf("  output_model=<path>       Output model file\n");
  std::printf("  output_vocab=<path>       Output vocab file\n");
  std::printf("  vocab_size=<int>          Target vocab size (default: 32000)\n");
  std::printf("  character_coverage=<float> Coverage 0.0-1.0 (default: 0.9995)\n");
  std::printf("  min_pair_freq=<int>       Min pair freq BPE (default: 2000)\n");
  std::printf("  num_iterations=<int>      Iterations Unigram (default: 10)\n");
}

struct Args {
  std::string input, model_type, output_model, output_vocab;
  bool has_input = false, has_type = false, has_model = false, has_vocab = false;
  int vocab_size = 32000;
  float coverage = 0.9995f;
  unsigned long long min_pair_freq = 2000;
};

}  // namespace

int main(int argc, char** argv) {
  std::printf("Tokenizer Trainer CLI v1.0\n==========================\n");
  if (argc < 2) {
    usage(argv[0]);
    return 0;
  }
  Args a;
  for (int i = 1; i < argc; ++i) {
    const char* arg = argv[i];
    const char* eq = std::strchr(arg, '=');
    if (!eq) continue;
    const std::string key(arg, eq - arg);
    const char* val = eq + 1;
    if (key == "input") { a.input = val; a.has_input = true; }
    else if (key == "model_type") { a.model_type = val; a.has_type = true; }
    else if (key == "output_model") { a.output_model = val; a.has_model = true; }
    else if (key == "output_vocab") { a.output_vocab = val; a.has_vocab = true; }
    else if (key == "vocab_size") a.vocab_size = std::atoi(val);
    else if (key == "character_coverage") a.coverage = (float)std::atof(val);
    else if (key == "min_pair_freq") a.min_pair_freq = std::strtoull(val, nullptr, 10);
  }
  if (!a.has_input || !a.has_type || !a.has_model || !a.has_vocab) {
    std::fprintf(stderr, "[ERROR] Missing required arguments\n\n");
    usage(argv[0]);
    return 1;
  }
  if (a.model_type != "bpe" && a.model_type != "unigram") {
    std::fprintf(stderr, "[ERROR] Invalid model_type. Must be 'bpe' or 'unigram'\n");
    return 1;
  }
  if (a.model_type == "unigram") {
    std::fprintf(stderr, "[ERROR] model_type=unigram is not supported by this MI355X BPE build\n");
    return 1;
  }
  std::printf("\n========== BPE Training ==========\n");
  std::printf("[CONFIG] Vocab Size: %d\n", a.vocab_size);
  std::printf("[CONFIG] Character Coverage: %.4f\n", a.coverage);
  std::printf("[CONFIG] Min Pair Freq: %llu\n", a.min_pair_freq);
  BPEConfig cfg;
  cfg.target_vocab_size = (size_t)a.vocab_size;
  cfg.unk_id = -1;
  cfg.character_coverage = a.coverage;
  cfg.min_pair_freq = a.min_pair_freq;
  Trainer* t = create_trainer(&cfg);
  std::printf("\n[STEP 1] Loading corpus from: %s\n", a.input.c_str());
  if (bpe_load_corpus(t, a.input.c_str()) != 0) {
    std::fprintf(stderr, "[ERROR] Failed to load corpus\n");
    bpe_trainer_destroy(t);
    return 255;
  }
  std::printf("\n[STEP 2] Training BPE model...\n");
  const int merges = bpe_train(t);
  if (merges < 0) {
    std::fprintf(stderr, "[ERROR] Training failed\n");
    bpe_trainer_destroy(t);
    return 255;
  }
  std::printf("[SUCCESS] Training completed with %d merges\n", merges);
  std::printf("\n[STEP 3] Saving model and vocabulary...\n");
  bpe_save(t, a.output_model.c_str(), a.output_vocab.c_str());
  std::printf("[SUCCESS] Saved to:\n  Model: %s\n  Vocab: %s\n", a.output_model.c_str(), a.output_vocab.c_str());
  bpe_trainer_destroy(t);
  std::printf("\n========== Training Complete ==========\n");
  return 0;
}
