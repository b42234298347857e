"""Read encoder on the GPU: the reference's Vectorizer / Preprocessor
(src/inference/vectorize.cpp:4-141, src/inference/preprocess.cpp:20-78) running the OpenVINO GRU model
(src/inference/fast_model.cpp, models/finetuned_sgn33-new-a-Apr6.xml) as one HIP kernel
(csrc/encoder_gru.hip) behind drm_encoder_* / drm_vectorize* (include/drm_hip.h).

`Encoder(path)` loads the reference's IR (.xml + .bin) or the compact .drmenc this repo ships
(DEFAULT_MODEL, written from the IR by drm_encoder_export)."""
import ctypes as C
import os

import numpy as np

from ._native import EncoderInfo, check, lib, ptr
from .rerank import pack_queries

DEFAULT_MODEL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "models",
                             "finetuned_sgn33-new-a-Apr6.drmenc")
MAX_LEN = 123         # Config::Inference::MAX_LEN (includes/utils/config.hpp:21)
BATCH_SIZE = 100      # Config::Inference::BATCH_SIZE (the IR's static batch; no effect on results)
MODEL_OUT_SIZE = 128  # Config::Inference::MODEL_OUT_SIZE


def _batch(seqs):
    if isinstance(seqs, tuple):  # (buf [n, stride] u8, lens [n] i32)
        buf, lens = seqs
        return np.ascontiguousarray(buf, dtype=np.uint8), np.ascontiguousarray(lens, dtype=np.int32)
    return pack_queries(seqs)


class Encoder:
    """drm_encoder: the GRU model resident on one GPU."""

    def __init__(self, model_path=DEFAULT_MODEL, device=0):
        h = C.c_void_p()
        check(lib().drm_encoder_load(str(model_path).encode(), int(device), C.byref(h)))
        self.handle = h.value
        self.path = str(model_path)

    @property
    def info(self):
        i = EncoderInfo()
        check(lib().drm_encoder_get_info(self.handle, C.byref(i)))
        return i

    def tokenize(self, seqs):
        """[n, 123] int32 model-input ids (0 padding, -1 = the reference's out-of-table read)."""
        buf, lens = _batch(seqs)
        out = np.empty((len(lens), MAX_LEN), dtype=np.int32)
        check(lib().drm_tokenize(self.handle, ptr(buf), ptr(lens), len(lens), buf.shape[1], ptr(out)))
        return out

    def vectorize(self, seqs, return_undefined=False):
        """[n, 128] float32 embeddings."""
        buf, lens = _batch(seqs)
        out = np.empty((len(lens), MODEL_OUT_SIZE), dtype=np.float32)
        und = C.c_int64(0)
        check(lib().drm_vectorize(self.handle, ptr(buf), ptr(lens), len(lens), buf.shape[1], ptr(out), C.byref(und)))
        return (out, und.value) if return_undefined else out

    def vectorize_device(self, d_seqs, d_lens, n, stride, d_out, stream=None):
        check(lib().drm_vectorize_device(self.handle, d_seqs.ptr, d_lens.ptr, int(n), int(stride), d_out.ptr,
                                         stream.handle if stream is not None else None))

    def flags(self):
        u, s = C.c_int64(0), C.c_int64(0)
        check(lib().drm_encoder_flags(self.handle, C.byref(u), C.byref(s)))
        return u.value, s.value

    def free(self):
        if self.handle:
            check(lib().drm_encoder_free(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


def export_encoder(model_path, out_path):
    """drm_encoder_export: IR (.xml) -> compact .drmenc (host only, no GPU)."""
    check(lib().drm_encoder_export(str(model_path).encode(), str(out_path).encode()))


class Preprocessor:
    """Preprocessor (includes/inference/preprocess.hpp:53-65) on the GPU tokenizer."""

    def __init__(self, encoder):
        self._enc = encoder

    def preprocess(self, seq, max_len=MAX_LEN):
        if max_len != MAX_LEN:
            raise ValueError("the model's input is [123, batch] (config.hpp:21)")
        s = seq.encode() if isinstance(seq, str) else bytes(seq)
        t = self._enc.tokenize([s])[0]
        return t[:min(max_len, len(s))]

    def preprocessBatch(self, seqs, max_len=MAX_LEN, verbose=False):  # noqa: N802 (reference name)
        return [self.preprocess(s, max_len) for s in seqs]


class Vectorizer:
    """Vectorizer (includes/inference/vectorize.hpp:15-50): vectorize(list of sequences) -> [n, 128]."""

    def __init__(self, model_path=DEFAULT_MODEL, batch_size=BATCH_SIZE, max_len=MAX_LEN,
                 model_out_size=MODEL_OUT_SIZE, device=0):
        if max_len != MAX_LEN or model_out_size != MODEL_OUT_SIZE:
            raise ValueError("the model is [123, batch] -> [batch, 128] (config.hpp:20-22)")
        self.batch_size = batch_size
        self.encoder = Encoder(model_path, device)

    def vectorize(self, input, verbose=False):  # noqa: A002 (reference name)
        return self.encoder.vectorize(input)
