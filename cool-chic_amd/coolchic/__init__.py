"""MI355X drop-in for Cool-chic's decode / forward hot path.

Mirrors the reference module surface (coolchic.enc.component.*, coolchic.decode, the
CCLIB decoder bindings) with the compute in libccmi's HIP kernels (include/ccmi.h).
Only the eval-mode (decode) forward is implemented; the training forward
(softround / noise quantisers, kron 2-D upsampling kernels, autograd) is the next
scope row and raises NotImplementedError.
"""
