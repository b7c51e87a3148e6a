"""firedancer_amd -- MI355X-native ed25519 batch signature verification for
Firedancer (drop-in for fd_ed25519_verify / fd_ed25519_verify_batch_single_msg).

The product is the C-ABI library firedancer_amd/_lib/libfd_ed25519_hip.so
(include/fd_ed25519_hip.h); `firedancer_amd.ed25519` is its Python mirror.
"""
import os

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
