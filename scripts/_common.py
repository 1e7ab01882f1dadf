"""Shared helpers for the measurement scripts.

Scripts never import oracle/ (test infrastructure only): inputs come from the
product's own generator (hbec_fill_splitmix, the SURVEY §8d splitmix64 stream)
and results are self-checked with the product's Encoder.Verify (a different
kernel from the one being timed).  Bit-exactness against the oracle is the
tests' job (tests/test_gpu_*.py)."""
from __future__ import annotations

import numpy as np
import torch

from hummingbird_amd import batch as B

HBEC_SEED = B.HBEC_SEED


def splitmix_bytes(n: int, seed: int = HBEC_SEED) -> np.ndarray:
    """The first n bytes of the splitmix64 stream seeded with `seed` (object 0
    of hbec_fill_splitmix with that base seed), e.g. config 4's size flags."""
    t = torch.empty((1, max(n, 1)), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(t, max(n, 1), base_seed=seed)
    return t.cpu().numpy()[0, :n].copy()


def objects_host(n: int, obj_len: int, first: int = 0) -> np.ndarray:
    """Synthetic objects first .. first+n-1 in host memory, [n, obj_len] uint8."""
    t = torch.empty((n, obj_len), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(t, obj_len, first=first)
    return t.cpu().numpy()


def verify_shards(enc, shards) -> bool:
    """Encoder.Verify over k+m host shards (runs on the GPU's verify path)."""
    return enc.Verify([np.ascontiguousarray(s) for s in shards])


def verify_stripe(enc, stripe: np.ndarray) -> bool:
    """Verify one ecSplit-layout stripe (k+m shards back to back)."""
    n = enc.Shards
    s = stripe.size // n
    return verify_shards(enc, [stripe[i * s:(i + 1) * s] for i in range(n)])
