"""Multi-GPU merge of aggregate shares.

Reports are sharded over ranks (one process per GPU); each rank folds its own
out shares on its GPU.  The only cross-GPU exchange is the per-prefix
aggregate share: one all-gather (RCCL over xGMI with the "nccl" backend)
into a rank-ordered buffer, then a GF(p) sum on the GPU
(``mastic_fold_shares``) — RCCL's integer sum is not field addition.
Mirrors ``Mastic.merge`` (poc/mastic.py:390-397).
"""
import ctypes

from . import _lib


def gather_shares(local, dist):
    """All-gather one uint8 tensor per rank into a rank-ordered flat tensor."""
    import torch
    world = dist.get_world_size()
    out = torch.empty(world * local.numel(), dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous())
    return out


def fold_on_gpu(m, gathered, world, n_elems):
    """merged[e] = sum_s gathered[s][e] mod p, computed by the HIP kernel."""
    import torch
    merged = torch.empty(n_elems * m.field.ENCODED_SIZE, dtype=torch.uint8, device=gathered.device)
    torch.cuda.synchronize()
    rc = _lib.lib().mastic_fold_shares(m._ctx, ctypes.c_void_p(gathered.data_ptr()), world, n_elems,
                                       ctypes.c_void_p(merged.data_ptr()))
    if rc != 0:
        raise _lib.MasticError(rc, "mastic_fold_shares failed")
    return merged


def merge_agg_shares(m, agg_share, dist):
    """Rank-local agg share (list of field elements, or its encode_vec bytes)
    -> job-wide agg share (uint8 device tensor in encode_vec order) on every rank."""
    import torch
    raw = bytes(agg_share) if isinstance(agg_share, (bytes, bytearray)) else m.field.encode_vec(agg_share)
    local = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    gathered = gather_shares(local, dist)
    return fold_on_gpu(m, gathered, dist.get_world_size(), len(raw) // m.field.ENCODED_SIZE)


def merge_field_shares(m, dist):
    """``merge`` callback for the sweep driver (heavy_hitters.compute_heavy_hitters):
    rank-local agg share -> job-wide agg share, both as lists of field elements."""
    def merge(agg_share):
        if len(agg_share) == 0:
            return agg_share
        merged = merge_agg_shares(m, agg_share, dist)
        return m.field.decode_vec(merged.cpu().numpy().tobytes())
    return merge
