"""The rejected single-pass 256v32 encoders (scripts/enc_variants.hip, a
measurement tool outside the library), byte-exact against the
oracle so that their A/B timings compare valid encoders.  Marker `variants`
(not `gpu`): `pytest -m variants` on a GPU box after scripts/build_variants.sh;
skipped without a HIP device or without scripts/libencvar.so."""
import ctypes
import os

import numpy as np
import pytest

import oracle_lib
from test_gpu_enc256v32 import mixed_blocks

torch = pytest.importorskip("torch")
tpf = pytest.importorskip("turbopfor_amd")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBVAR = os.path.join(ROOT, "scripts", "libencvar.so")
pytestmark = [pytest.mark.variants,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="no HIP device visible"),
              pytest.mark.skipif(not os.path.exists(LIBVAR), reason="scripts/libencvar.so not built (scripts/build_variants.sh)")]
DEV = "cuda:0"


def encvar(mode, vals, nb):
    tpf.lib()  # the library first (libencvar links it)
    V = ctypes.CDLL(LIBVAR)
    V.encvar_workspace_size.restype = ctypes.c_size_t
    V.encvar_workspace_size.argtypes = [ctypes.c_uint64]
    V.encvar_launch.restype = ctypes.c_int
    V.encvar_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    cap = int(tpf.lib().tpf_p4enc256v32_bound(nb))
    out = torch.zeros(cap, dtype=torch.uint8, device=DEV)
    offs = torch.empty(nb + 1, dtype=torch.int64, device=DEV)
    wsb = int(V.encvar_workspace_size(nb))
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=DEV)
    rc = V.encvar_launch(mode, vals.data_ptr(), nb, out.data_ptr(), cap, offs.data_ptr(), ws.data_ptr(), wsb,
                         torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc
    return out, offs


@pytest.mark.parametrize("mode", [4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 16 + 64 + 1024])
@pytest.mark.parametrize("nb", [1, 31, 33, 1000, 20_000])
def test_encoder_variants_vs_oracle(mode, nb):
    """4 = look-back encoder forced onto its gated two-pass fallback, 5/6/7 =
    4/6/8 blocks per wave in fixed slots, 8-11 = per-wave arenas, 12 = its
    default arena, 13-15 = two-pass with nt / sc1 value loads, 16/17 =
    two-pass on a persistent grid, 16+64+1024 = pipelined (64-item chunks, lag 1).
    Ragged last tiles; 20,000 blocks = 625+ tiles (look-backs longer than one poll)."""
    blocks = mixed_blocks(nb, nb + mode)
    exp_packed, exp_off = oracle_lib.enc256v32_batch(blocks)
    vals = torch.from_numpy(np.ascontiguousarray(blocks, dtype=np.uint32).view(np.int32)).to(DEV)
    out, offs = encvar(mode, vals, nb)
    np.testing.assert_array_equal(offs.cpu().numpy().astype(np.uint64), exp_off)
    np.testing.assert_array_equal(out.cpu().numpy()[:int(offs[-1].item())], exp_packed)
