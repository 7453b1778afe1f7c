"""BERT-base gradient shapes and backward-GEMM schedule (BASELINE.json config 5).

The reference has no transformer; config 5 asks for "BERT-base layer gradients bf16: backward MFMA GEMM
overlapped with compressed all-reduce on a side HIP stream". This module provides exactly that workload:
the parameter tensors of BERT-base (uncased: vocab 30522, hidden 768, 12 layers, FFN 3072, 512 positions),
grouped into per-layer gradient buckets in backward order, and the list of backward GEMMs (bwd-data +
bwd-weight of the four projections of every encoder layer) for ``tokens = batch x seq`` rows.
"""
from __future__ import annotations

from dataclasses import dataclass

HIDDEN, LAYERS, FFN, VOCAB, POS, TYPES = 768, 12, 3072, 30522, 512, 2


@dataclass
class Bucket:
    name: str
    tensors: list  # (name, shape)

    @property
    def numel(self):
        n = 0
        for _, s in self.tensors:
            k = 1
            for d in s:
                k *= d
            n += k
        return n


def encoder_layer_tensors(i: int, h: int = HIDDEN, f: int = FFN):
    p = f"encoder.layer.{i}."
    return [(p + "attention.self.qkv.weight", (h, 3 * h)), (p + "attention.self.qkv.bias", (3 * h,)),
            (p + "attention.output.dense.weight", (h, h)), (p + "attention.output.dense.bias", (h,)),
            (p + "attention.output.LayerNorm.weight", (h,)), (p + "attention.output.LayerNorm.bias", (h,)),
            (p + "intermediate.dense.weight", (h, f)), (p + "intermediate.dense.bias", (f,)),
            (p + "output.dense.weight", (f, h)), (p + "output.dense.bias", (h,)),
            (p + "output.LayerNorm.weight", (h,)), (p + "output.LayerNorm.bias", (h,))]


def gradient_buckets(layers: int = LAYERS):
    """Buckets in the order their gradients become ready during backward (pooler, layers L-1..0, embeddings)."""
    out = [Bucket("pooler", [("pooler.dense.weight", (HIDDEN, HIDDEN)), ("pooler.dense.bias", (HIDDEN,))])]
    for i in reversed(range(layers)):
        out.append(Bucket(f"layer{i}", encoder_layer_tensors(i)))
    out.append(Bucket("embeddings", [("embeddings.word_embeddings.weight", (VOCAB, HIDDEN)),
                                     ("embeddings.position_embeddings.weight", (POS, HIDDEN)),
                                     ("embeddings.token_type_embeddings.weight", (TYPES, HIDDEN)),
                                     ("embeddings.LayerNorm.weight", (HIDDEN,)),
                                     ("embeddings.LayerNorm.bias", (HIDDEN,))]))
    return out


def num_params(layers: int = LAYERS) -> int:
    return sum(b.numel for b in gradient_buckets(layers))


def layer_backward_gemms(tokens: int, h: int = HIDDEN, f: int = FFN):
    """(name, M, N, K, a_t, b_t) of the backward GEMMs of one encoder layer, in execution order:
    FFN-out, FFN-in, attention-out, QKV; each as bwd-data (dX = dY·Wᵀ) then bwd-weight (dW = Xᵀ·dY)."""
    lin = [("ffn_out", f, h), ("ffn_in", h, f), ("attn_out", h, h), ("qkv", h, 3 * h)]
    out = []
    for name, fin, fout in lin:
        out.append((name + ".dgrad", tokens, fin, fout, False, True))    # [T,fout]·[fin,fout]ᵀ
        out.append((name + ".wgrad", fin, fout, tokens, True, False))    # [T,fin]ᵀ·[T,fout]
    return out


def layer_backward_flops(tokens: int) -> float:
    return sum(2.0 * M * N * K for _, M, N, K, _, _ in layer_backward_gemms(tokens))
