/* shredword_encode.h — C ABI of the MI355X BPE encoder (libtrainer.so).
 *
 * Reads the trainer's on-disk formats and applies a trained merge list to text on the GPU.
 *   .model  M records of three native int32 (first, second, new_id = 256 + m), written by the
 *           reference's bpe_save (shredword/csrc/bpe/bpe.cpp:419-427);
 *   .vocab  256 + M records "<token bytes> <freq>\n" (bpe.cpp:416-418), token m = concatenation
 *           of its two operands' bytes (bpe.cpp:400-408).
 * The reference ships no loader or encoder for these files; the encoding is defined as the
 * trainer's own merge application replayed on new text: words are the maximal runs of bytes
 * outside "\t\r\n " (the strtok split of bpe.cpp:143-153), each byte becomes its symbol id
 * (bpe.cpp:154-180; bytes the trainer's coverage rule dropped become unk_id), and merge m is
 * applied to every word left to right without overlap (bpe.cpp:265-296) for m = 0, 1, ... .
 * Encoding the training corpus therefore reproduces the trainer's final segmentation, and the
 * per-id counts of the result equal the .vocab frequency column.
 *
 * Plain pointers and sizes only.  The handle owns device memory on one GPU; it is not
 * thread-safe.  Every entry point needs a HIP device: there is no CPU encoder.
 */
#ifndef SHREDWORD_ENCODE_H
#define SHREDWORD_ENCODE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ShredEncoder ShredEncoder;

/* Longest word the encoder accepts (bytes); a longer word fails the call with -3. */
#define SHRED_ENCODE_MAX_WORD 1024

/* merges: num_merges triples (first, second, new_id) as in a .model file; new_id must be 256 + m
 * and first/second must be ids < new_id (or the call fails).  byte_map: 256 symbol ids (byte b
 * -> byte_map[b]) or NULL for the identity.  Returns NULL on invalid input or without a device
 * (the reason goes to stderr). */
ShredEncoder* shred_encoder_create(const int32_t* merges, size_t num_merges, const int32_t* byte_map,
                                   int device);

/* Loads a .model file.  With a .vocab path (may be NULL), bytes whose .vocab frequency is 0 and
 * that no merge uses map to unk_id (the trainer's coverage rule, recovered from its outputs);
 * without one the byte map is the identity. */
ShredEncoder* shred_encoder_load(const char* model_path, const char* vocab_path, int32_t unk_id, int device);

void shred_encoder_destroy(ShredEncoder* enc);

/* num_merges and the 256-entry byte map of an encoder (either pointer may be NULL). */
int shred_encoder_info(const ShredEncoder* enc, size_t* num_merges, int32_t* byte_map);

/* Encodes n bytes of host text into host ids.  Returns the number of ids written (<= the number
 * of non-delimiter bytes, so cap >= n always suffices), or -1 on a bad argument / device error,
 * -2 when cap is smaller than the result, -3 when a word exceeds SHRED_ENCODE_MAX_WORD. */
int64_t shred_encode(ShredEncoder* enc, const uint8_t* text, size_t n, int32_t* out, size_t cap);

/* The same on device buffers (text: n bytes, out: cap >= n int32, both on the encoder's device),
 * queued on `stream` (a hipStream_t, NULL = the encoder's own) and synchronised before return.
 * Same return values; kernel_ms (may be NULL) receives the device time of the encode passes. */
int64_t shred_encode_device(ShredEncoder* enc, const void* text, size_t n, void* out, size_t cap,
                            void* stream, double* kernel_ms);

/* Concatenates the bytes of n token ids into out (cap bytes).  Returns the byte count needed
 * (nothing is written past cap), or -1 for an id outside [0, 256 + num_merges).  Host only. */
int64_t shred_decode(const ShredEncoder* enc, const int32_t* ids, size_t n, uint8_t* out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* SHREDWORD_ENCODE_H */
