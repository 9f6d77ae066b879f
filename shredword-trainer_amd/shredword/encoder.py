"""BPEEncoder — applies a trained ``.model`` to text on the GPU.

The reference writes ``.model`` / ``.vocab`` (shredword/csrc/bpe/bpe.cpp:388-432) but ships no
loader or encoder for them.  This one defines encoding as the trainer's own merge application
replayed on new text (include/shredword_encode.h): words are the runs of bytes outside
``"\\t\\r\\n "``, bytes map to symbol ids (bytes the trainer's coverage rule dropped map to
``unk_id`` when the ``.vocab`` is given), and the merges apply in training order.  Encoding the
training corpus reproduces the trainer's segmentation, so the id counts equal the ``.vocab``
frequencies.  Every call runs the gfx950 kernels through libtrainer.so; there is no CPU path.
"""
import atexit
import ctypes
import weakref

import numpy as np

from .cbase import lib

MAX_WORD = 1024  # SHRED_ENCODE_MAX_WORD

# Encoders still alive at interpreter exit are destroyed while the HIP runtime is up (a destructor
# that ran after the runtime's own teardown would free its device memory twice).
_LIVE = weakref.WeakSet()


@atexit.register
def _destroy_live():
    for e in list(_LIVE):
        e.destroy()


class BPEEncoder:
    def __init__(self, model_path: str, vocab_path: str = None, unk_id: int = 0, device: int = 0):
        self.enc = lib.shred_encoder_load(model_path.encode("utf-8"),
                                          vocab_path.encode("utf-8") if vocab_path else None,
                                          int(unk_id), int(device))
        self.device = int(device)
        if not self.enc:
            raise RuntimeError(f"Failed to create the encoder for {model_path} (see stderr; a GPU is required)")
        _LIVE.add(self)

    @classmethod
    def from_merges(cls, merges, byte_map=None, device: int = 0):
        """merges: (M, 3) int32 array of (first, second, 256 + m) as in a .model file."""
        m = np.ascontiguousarray(np.asarray(merges, dtype=np.int32).reshape(-1, 3))
        bm = None if byte_map is None else np.ascontiguousarray(np.asarray(byte_map, dtype=np.int32))
        if bm is not None and bm.shape != (256,):
            raise ValueError("byte_map must hold 256 ids")
        self = cls.__new__(cls)
        self.enc = lib.shred_encoder_create(m.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), m.shape[0],
                                            None if bm is None else bm.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                            int(device))
        self.device = int(device)
        if not self.enc:
            raise RuntimeError("Failed to create the encoder (invalid merges or no GPU; see stderr)")
        _LIVE.add(self)
        return self

    @property
    def num_merges(self) -> int:
        n = ctypes.c_size_t()
        lib.shred_encoder_info(self.enc, ctypes.byref(n), None)
        return n.value

    @property
    def byte_map(self) -> np.ndarray:
        out = np.empty(256, dtype=np.int32)
        lib.shred_encoder_info(self.enc, None, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        return out

    @staticmethod
    def _check(r: int) -> int:
        if r == -3:
            raise ValueError(f"a word is longer than {MAX_WORD} bytes")
        if r < 0:
            raise RuntimeError(f"encode failed (code {r})")
        return r

    def encode(self, text) -> np.ndarray:
        """bytes / str / uint8 array -> int32 ids of every word, in text order."""
        if isinstance(text, str):
            text = text.encode("utf-8")
        buf = np.frombuffer(text, dtype=np.uint8) if isinstance(text, (bytes, bytearray, memoryview)) \
            else np.ascontiguousarray(text, dtype=np.uint8)
        out = np.empty(max(1, buf.size), dtype=np.int32)
        r = self._check(lib.shred_encode(self.enc, buf.ctypes.data, buf.size, out.ctypes.data, out.size))
        return out[:r].copy()

    def encode_device(self, text, out=None, stream=None):
        """text: 1-D uint8 torch tensor on the encoder's GPU -> (int32 tensor view of the ids,
        device milliseconds of the encode kernels)."""
        import torch
        if text.dtype != torch.uint8 or text.dim() != 1 or not text.is_cuda or not text.is_contiguous():
            raise ValueError("text must be a contiguous 1-D uint8 CUDA tensor")
        if text.device.index != self.device:
            raise ValueError(f"text is on {text.device}, the encoder on cuda:{self.device}")
        n = text.numel()
        if out is None:
            out = torch.empty(max(1, n), dtype=torch.int32, device=text.device)
        elif out.dtype != torch.int32 or not out.is_cuda or not out.is_contiguous() or out.device != text.device:
            raise ValueError("out must be a contiguous int32 tensor on the text's device")
        ms = ctypes.c_double()
        st = stream if stream is not None else torch.cuda.current_stream(text.device).cuda_stream
        r = self._check(lib.shred_encode_device(self.enc, text.data_ptr(), n, out.data_ptr(), out.numel(),
                                                ctypes.c_void_p(st), ctypes.byref(ms)))
        return out[:r], ms.value

    def decode(self, ids) -> bytes:
        """Concatenated bytes of the ids (whitespace between words is not restored)."""
        a = np.ascontiguousarray(ids, dtype=np.int32)
        need = lib.shred_decode(self.enc, a.ctypes.data, a.size, None, 0)
        if need < 0:
            raise ValueError("id outside the vocabulary")
        out = np.empty(max(1, need), dtype=np.uint8)
        lib.shred_decode(self.enc, a.ctypes.data, a.size, out.ctypes.data, out.size)
        return out[:need].tobytes()

    def destroy(self):
        if getattr(self, "enc", None):
            lib.shred_encoder_destroy(self.enc)
            self.enc = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.destroy()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass
