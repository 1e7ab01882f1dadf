"""hummingbird_amd — MI355X-native (gfx950) erasure coding for Hummingbird's
`hec` EC policy: the GF(2^8) Reed-Solomon encode / reconstruct behind
objectserver/ecutils.go, as HIP kernels behind a C ABI (include/hbec.h).

Modules:
  reedsolomon — the klauspost Encoder surface (New / Encode / Reconstruct / ReconstructData)
  ecutils     — ecSplit / ecReconstruct / ecGlue / ecShardLength / parseECScheme / rangeChunkAlign
  batch       — device-resident batches on torch tensors (the bench hot path)
  build       — hipcc build of libhbec.so
"""
from .reedsolomon import New, Encoder  # noqa: F401

__all__ = ["New", "Encoder"]
