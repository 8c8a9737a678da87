"""Multi-GPU merge of aggregate shares.

Reports are sharded over ranks (one process per GPU); each rank folds its own
out shares on its GPU.  The only cross-GPU exchange is the per-prefix
aggregate share: one all-gather over xGMI into a rank-ordered buffer, then a
GF(p) sum on the GPU (``k_fold_shares``) — RCCL's integer sum is not field
addition.  Mirrors ``Mastic.merge`` (poc/mastic.py:390-397).

The product path is :class:`CommMerge`: the library owns the RCCL
communicator (``mastic_comm_init``) and does fold, all-gather and GF(p) merge
in HBM in one call (``mastic_aggregate_merged``); no PyTorch is involved, and
the communicator id crosses processes by whatever channel the caller has
(:func:`exchange_unique_id` takes any broadcast callable).

The torch forms below (``gather_shares`` / :class:`SweepMerge`) keep the
same fold and merge kernels but let a ``torch.distributed`` group move the
shares: a ``gloo`` group is how several ranks share ONE GPU in the one-GPU
rehearsals (RCCL refuses two ranks on one device).
"""
import ctypes

from . import _lib


def exchange_unique_id(m, rank: int, broadcast):
    """The communicator id on every rank: rank 0 creates it
    (``mastic_comm_unique_id``) and ``broadcast(obj_or_None) -> obj`` hands
    it to the others (e.g. a ``torch.distributed.broadcast_object_list``
    wrapper, a file or a socket)."""
    uid = m.comm_unique_id() if rank == 0 else None
    return bytes(broadcast(uid))


class CommMerge:
    """Per-level merge for the sweep driver over the library's own RCCL
    communicator.  ``total`` folds both aggregators' out shares on this rank's
    GPU, all-gathers them across the ranks and sums the 2 x world shares mod p
    (the collector's ``unshard`` merge, mastic.py:399-411, of the job-wide agg
    shares), all inside ``mastic_aggregate_merged``; only the final aggregate
    reaches the host.  Calling the object maps a list of field elements (one
    aggregator's rank-local agg share) to the job-wide list."""

    def __init__(self, m, nranks: int = None, rank: int = None, unique_id: bytes = None):
        self.m = m
        if nranks is not None and m.comm_info()[0] == 1 and nranks > 1:
            m.comm_init(nranks, rank, unique_id)

    def total(self, n_elems, valid=None, have_results=True) -> bytes:
        if n_elems == 0:
            return b""
        return self.m.aggregate_merged((0, 1), n_elems, None if not have_results else valid,
                                       zeros=not have_results)

    def __call__(self, agg_share):
        m = self.m
        if len(agg_share) == 0:
            return agg_share
        raw = bytes(agg_share) if isinstance(agg_share, (bytes, bytearray)) else m.field.encode_vec(agg_share)
        merged = m.merge_host(raw, 1, len(raw) // m.field.ENCODED_SIZE)
        return m.field.decode_vec(merged)


def _current_stream_handle():
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def gather_shares(local, dist):
    """All-gather one uint8 tensor per rank into a rank-ordered flat tensor
    (RCCL over xGMI for device tensors under the "nccl" backend; a "gloo"
    group, e.g. several ranks sharing one GPU in a test, gathers host copies)."""
    import torch
    if local.is_cuda and dist.get_backend() == "gloo":
        return gather_shares(local.cpu(), dist).to(local.device)
    world = dist.get_world_size()
    out = torch.empty(world * local.numel(), dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous())
    return out


def fold_on_gpu(m, shares, n_shares, n_elems):
    """merged[e] = sum_s shares[s][e] mod p, computed by the HIP kernel.
    ``shares`` is a uint8 device tensor of n_shares x n_elems encode_vec
    elements, written on torch's current stream."""
    import torch
    merged = torch.empty(n_elems * m.field.ENCODED_SIZE, dtype=torch.uint8, device=shares.device)
    rc = _lib.lib().mastic_fold_shares(m._ctx, ctypes.c_void_p(shares.data_ptr()), n_shares, n_elems,
                                       ctypes.c_void_p(merged.data_ptr()), _current_stream_handle())
    if rc != 0:
        raise _lib.MasticError(rc, "mastic_fold_shares failed")
    return merged


def aggregate_to_tensor(m, agg_id, n_elems, valid=None, out=None):
    """The GPU fold of agg_id's last prep_init out shares, left in HBM as a
    uint8 tensor (``mastic_aggregate_device_on_stream``).  The library orders the fold
    after the work queued on torch's current stream (the tensor's allocation
    or fill) by an event."""
    import numpy as np
    import torch
    if out is None:
        out = torch.empty(n_elems * m.field.ENCODED_SIZE, dtype=torch.uint8, device="cuda")
    v = None if valid is None else np.ascontiguousarray(np.asarray(valid, dtype=np.uint8))
    rc = _lib.lib().mastic_aggregate_device_on_stream(m._ctx, agg_id, _lib.buf(v),
                                                      ctypes.c_void_p(out.data_ptr()), _current_stream_handle())
    if rc != 0:
        raise _lib.MasticError(rc, "mastic_aggregate_device_on_stream failed")
    return out


def merge_agg_shares(m, agg_share, dist):
    """Rank-local agg share (a uint8 device tensor, its encode_vec bytes, or a
    list of field elements) -> job-wide agg share (uint8 device tensor in
    encode_vec order) on every rank."""
    import torch
    if isinstance(agg_share, torch.Tensor):
        local = agg_share
    else:
        raw = bytes(agg_share) if isinstance(agg_share, (bytes, bytearray)) else m.field.encode_vec(agg_share)
        local = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    gathered = gather_shares(local, dist)
    return fold_on_gpu(m, gathered, dist.get_world_size(), local.numel() // m.field.ENCODED_SIZE)


class SweepMerge:
    """Per-level merge for the sweep driver (heavy_hitters.compute_heavy_hitters)
    on N ranks.  ``total`` folds both aggregators' out shares on this rank's
    GPU into one device buffer [agg 0 | agg 1], all-gathers it (one RCCL call
    per level), and sums the 2 x world shares mod p on the GPU: that is the
    collector's ``unshard`` merge (mastic.py:399-411) of the job-wide agg
    shares, so only the final aggregate (len(prefixes) x (1 + OUTPUT_LEN)
    elements) comes back to the host for the pruning decision.

    Calling the object maps a list of field elements to the job-wide list (the
    per-share form, kept for drivers that merge shares one by one)."""

    def __init__(self, m, dist):
        self.m = m
        self.dist = dist

    def total(self, n_elems, valid=None, have_results=True) -> bytes:
        import torch
        m = self.m
        enc = m.field.ENCODED_SIZE
        if n_elems == 0:
            return b""
        if have_results:
            # k_fold writes every element; the fold is ordered after this
            # allocation's stream by an event (mastic_aggregate_device_on_stream)
            local = torch.empty(2 * n_elems * enc, dtype=torch.uint8, device="cuda")
            for agg_id in range(2):
                aggregate_to_tensor(m, agg_id, n_elems, valid, out=local[agg_id * n_elems * enc:])
        else:  # a rank with no reports contributes zero shares (agg_init)
            local = torch.zeros(2 * n_elems * enc, dtype=torch.uint8, device="cuda")
        gathered = gather_shares(local, self.dist)
        merged = fold_on_gpu(m, gathered, 2 * self.dist.get_world_size(), n_elems)
        return merged.cpu().numpy().tobytes()

    def __call__(self, agg_share):
        if len(agg_share) == 0:
            return agg_share
        merged = merge_agg_shares(self.m, agg_share, self.dist)
        return self.m.field.decode_vec(merged.cpu().numpy().tobytes())


def merge_field_shares(m, dist):
    """``merge`` for the sweep driver: a :class:`SweepMerge`."""
    return SweepMerge(m, dist)
