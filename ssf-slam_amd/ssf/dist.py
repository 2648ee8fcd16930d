"""Multi-GPU layout: one process per GPU, sequences sharded across ranks.

The path shards naturally -- frames are independent for the mask and the features, and a
sequence's registration chain is serial (warm start, src/lidarOdometry_onlyPC.cpp:164,251-252)
-- so every rank owns whole sequences and there is no data-path collective.  The one exchange
step is an all-gather of the per-frame 6-DoF poses (RCCL over xGMI on the GPU, gloo in the
CPU tests), done once per batch: it is latency-bound (B x 14 doubles per rank), not
bandwidth-bound, so it is never split into smaller messages.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def sequence_shard(n_sequences: int, world: int, rank: int) -> range:
    """Contiguous block of sequence ids owned by `rank` (sizes differ by at most one)."""
    base, extra = divmod(n_sequences, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def pose_record(pose_abs: torch.Tensor, mask_out: torch.Tensor | None = None) -> torch.Tensor:
    """Per-frame record exchanged between ranks: accumulated registration pose [q xyzw, t]
    (7 doubles) and, if given, the SSF Kabsch pose [t, q xyzw] (7 doubles)."""
    parts = [pose_abs.to(torch.float64)]
    if mask_out is not None:
        parts.append(mask_out[:, 0:7].to(torch.float64))
    return torch.cat(parts, 1).contiguous()


def gather_pose_records(records, group=None) -> torch.Tensor:
    """Deferred exchange: the records of K steps ([K] x [n, k], one per step, each from
    pose_record) stacked and all-gathered in ONE collective -> [K, world * n, k], step-major,
    ranks in order within a step.  Used at the end of a run (or every K steps) so that no step
    of the pipeline waits on its streams for a collective (once per batch or
    at the end of a sequence)."""
    stack = torch.stack(list(records), 0).contiguous()          # [K, n, k]
    K, n, k = stack.shape
    allr = gather_poses(stack.view(K, n * k), group)             # [world * K, n * k]
    world = allr.shape[0] // K
    return allr.view(world, K, n, k).transpose(0, 1).reshape(K, world * n, k)


def gather_sequence_records(records: torch.Tensor, n_sequences: int, group=None) -> torch.Tensor:
    """Strong-scaling exchange (BASELINE configs[3]: a fixed set of n_sequences sharded over the
    ranks by sequence_shard): this rank's per-frame records [F, B_r, k] (B_r = its shard size,
    frames in order) -> [F, n_sequences, k], sequences in id order, in ONE all-gather.  Shards
    may differ in size by one, so every rank pads to the largest shard (NaN rows) before the
    collective and the pads are dropped after it."""
    F, b, k = records.shape
    if not records.dtype.is_floating_point:
        raise TypeError(f"sequence records must be floating point (NaN pads), got {records.dtype}")
    if not dist.is_available() or not dist.is_initialized():
        if b != n_sequences:
            raise ValueError(f"{b} sequences on a single rank, expected {n_sequences}")
        return records
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if b != len(sequence_shard(n_sequences, world, rank)):
        raise ValueError("records do not match this rank's sequence shard")
    # the concatenation below puts rank r's rows at sequence_shard(.., r): that is the id order
    # only because the shards are contiguous, in rank order, and cover every id once
    shards = [sequence_shard(n_sequences, world, r) for r in range(world)]
    if [i for sh in shards for i in sh] != list(range(n_sequences)):
        raise AssertionError("sequence_shard must give contiguous id-ordered shards")
    bmax = -(-n_sequences // world)
    pad = torch.full((F, bmax, k), float("nan"), dtype=records.dtype, device=records.device)
    pad[:, :b] = records
    allr = gather_poses(pad.view(F, bmax * k), group).view(world, F, bmax, k)
    parts = [allr[r, :, :len(shards[r])] for r in range(world)]
    return torch.cat(parts, 1)


def gather_poses(local: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather equal-shaped per-rank pose records -> [world * n, k] in rank order."""
    if not dist.is_available() or not dist.is_initialized():
        return local
    if local.is_cuda and dist.get_backend(group) == "gloo":     # gloo gathers host tensors
        return gather_poses(local.cpu(), group).to(local.device)
    world = dist.get_world_size(group)
    bufs = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(bufs, local.contiguous(), group=group)
    return torch.cat(bufs, 0)
