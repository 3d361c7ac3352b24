"""Gradient tensor shapes of the model configs named in BASELINE.json.

The reference allreduces one flat float vector per round (AllreduceWorker.scala:171-178);
a data-parallel trainer allreduces a model's gradient set. These are the exact parameter
shapes of the two BASELINE models (architecture only; values are synthetic):

  resnet50   - torchvision ResNet-50 (25.56 M parameters, 161 tensors incl. BN affine)
  llama3_8b  - Llama-3-8B (8.03 B parameters, 291 tensors; 16.06 GB of bf16 gradients)
  flat256m   - one 256 MiB bf16 buffer (BASELINE config 3)
"""
from __future__ import annotations

from typing import Callable


def resnet50_shapes() -> list[tuple[str, tuple[int, ...]]]:
    shapes: list[tuple[str, tuple[int, ...]]] = []

    def conv_bn(name: str, cout: int, cin: int, k: int) -> None:
        shapes.append((f"{name}.weight", (cout, cin, k, k)))
        shapes.append((f"{name}.bn.weight", (cout,)))
        shapes.append((f"{name}.bn.bias", (cout,)))

    conv_bn("conv1", 64, 3, 7)
    cin = 64
    for li, (width, blocks) in enumerate([(64, 3), (128, 4), (256, 6), (512, 3)], start=1):
        for b in range(blocks):
            pre = f"layer{li}.{b}"
            conv_bn(f"{pre}.conv1", width, cin, 1)
            conv_bn(f"{pre}.conv2", width, width, 3)
            conv_bn(f"{pre}.conv3", width * 4, width, 1)
            if b == 0:
                conv_bn(f"{pre}.downsample", width * 4, cin, 1)
            cin = width * 4
    shapes.append(("fc.weight", (1000, 2048)))
    shapes.append(("fc.bias", (1000,)))
    return shapes


def llama3_8b_shapes(layers: int = 32) -> list[tuple[str, tuple[int, ...]]]:
    d, kv, ff, vocab = 4096, 1024, 14336, 128256
    shapes: list[tuple[str, tuple[int, ...]]] = [("tok_embeddings.weight", (vocab, d))]
    for i in range(layers):
        p = f"layers.{i}"
        shapes += [
            (f"{p}.attention_norm.weight", (d,)),
            (f"{p}.attention.wq.weight", (d, d)),
            (f"{p}.attention.wk.weight", (kv, d)),
            (f"{p}.attention.wv.weight", (kv, d)),
            (f"{p}.attention.wo.weight", (d, d)),
            (f"{p}.ffn_norm.weight", (d,)),
            (f"{p}.feed_forward.w1.weight", (ff, d)),
            (f"{p}.feed_forward.w3.weight", (ff, d)),
            (f"{p}.feed_forward.w2.weight", (d, ff)),
        ]
    shapes += [("norm.weight", (d,)), ("output.weight", (vocab, d))]
    return shapes


def flat_shapes(mib: int = 256, elem_bytes: int = 2) -> list[tuple[str, tuple[int, ...]]]:
    return [("flat", ((mib << 20) // elem_bytes,))]


GRAD_SETS: dict[str, Callable[[], list[tuple[str, tuple[int, ...]]]]] = {
    "resnet50": resnet50_shapes,
    "llama3_8b": llama3_8b_shapes,
    "flat256m": flat_shapes,
}


def gradient_shapes(name: str) -> list[tuple[str, tuple[int, ...]]]:
    try:
        return GRAD_SETS[name]()
    except KeyError:
        raise ValueError(f"unknown gradient set {name!r}; choose from {sorted(GRAD_SETS)}") from None


def numel(shape: tuple[int, ...]) -> int:
    n = 1
    for s in shape:
        n *= s
    return n
