// The 13 Unigram symbols that the reference's ctypes layer binds at import time
// (shredword/cbase.py:59-71).  Unigram training is outside the BPE hot path this build replaces
// (SURVEY.md §2 #7), so each stub reports failure; BPETrainer users are unaffected, and
// UnigramTrainer(...) raises RuntimeError("Failed to create Unigram trainer") as the reference
// does when trainerCreate returns NULL (trainer.py:46).
#include <cstdio>

#include "../../../include/shredword_bpe.h"

namespace {
void unsupported(const char* fn) {
  std::fprintf(stderr, "[ERROR]\t %s: the Unigram trainer is not part of this MI355X BPE build\n", fn);
}
}  // namespace

extern "C" {
void* trainerCreate(int, float, int, int) { unsupported("trainerCreate"); return nullptr; }
void trainerDestroy(void*) {}
int addTextToTrainer(void*, const char*) { unsupported("addTextToTrainer"); return 0; }
int preprocessTexts(void*) { unsupported("preprocessTexts"); return 0; }
int extractInitialSubwords(void*) { unsupported("extractInitialSubwords"); return 0; }
float computeLoss(void*, char**, int) { unsupported("computeLoss"); return 0.0f; }
double computeTokenLoss(void*, const char*, char**, int) { unsupported("computeTokenLoss"); return 0.0; }
int pruneVocabStep(void*, char**, int, double) { unsupported("pruneVocabStep"); return 0; }
int updateTokenScores(void*, char**, int) { unsupported("updateTokenScores"); return 0; }
int trainUnigram(void*, char**, int, int) { unsupported("trainUnigram"); return 0; }
int getVocab(void*, char***, double**, int*) { unsupported("getVocab"); return 0; }
int saveVocab(void*, const char*) { unsupported("saveVocab"); return 0; }
int loadVocab(void*, const char*) { unsupported("loadVocab"); return 0; }
}
