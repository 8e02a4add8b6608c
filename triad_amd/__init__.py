"""triad_amd: MI355X-native (gfx950 / CDNA4) dense tri-modal contrastive training path.

Drop-in for SajayR/TRIAD's src/model.py encoder/projector API and src/train.py
step; the hot path (projection heads, fused token-similarity / max-mean
aggregation / InfoNCE + regularisers and their backward) runs as hand-written
HIP kernels from libtriad_hip.so.
"""
__version__ = "0.1.0"

# Importing the package changes no process-wide state. The vendor-BLAS choice for the GEMMs torch
# still runs (rocBLAS, not hipBLASLt's stream-K kernels) is an explicit opt-in:
# `triad_amd.blas.configure()`, which TriadTrainer and bench.py call (triad_amd/blas.py).
