"""Data parallel on batch, one process per GPU (torch.distributed; backend "nccl" = RCCL on
ROCm, gloo for CPU tests).  SURVEY.md 8(e):

* every rank trains its own shard of the global batch with replicated weights;
* the flat gradient buffer (8.70 M fp32 = 34.8 MB at c2) is summed in two buckets: the top
  LSTM layer + decoder heads (74 % of it at c2, final once the top layer's weight gradients
  are done) on a communication stream while the lower layers' BPTT runs, the rest (bottom
  layer + encoder) in optimizer_step;
* the masked-mean denominators use the all-reduced valid-frame count, so each rank's
  gradient is its exact share of the global masked mean and the SUM over ranks equals the
  single-GPU gradient of the global batch (no 1/world rescale, exact for unequal lengths);
* the loss scalars ride along so every rank takes the same non-finite-skip decision and
  clips with the same global norm;
* eps and the dropout masks are drawn from counter-based streams indexed by (global utterance,
  frame), so the sampled noise is independent of the rank count; this needs every rank's batch
  padded to the same T -- the global batch's longest utterance (utils/data_io.py _batched does
  that), exactly the single-process batch's padding.
"""
import torch
import torch.distributed as dist


def attach(engine, rank, world, batch_per_rank, group=None):
    """Make a VAEEngine data-parallel: shard offset, process group, identical weights."""
    engine.process_group = group
    engine.world = world
    engine.rank = rank
    # first global utterance of this shard; re-derived from every batch's own size in
    # VAEEngine.forward (rank * B), so the loader's batch size -- not a config value -- decides
    engine.global_offset = rank * batch_per_rank
    broadcast_params(engine.flat, group)
    return engine


def broadcast_params(flat, group=None):
    dist.broadcast(flat, src=0, group=group)


def allreduce_step(grad_flat, loss3, group=None):
    """Sum the flat gradient buffer and the [kld, recon, total] loss shares over ranks."""
    dist.all_reduce(grad_flat, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(loss3, op=dist.ReduceOp.SUM, group=group)


def allreduce_grad_bucket(buf, group=None):
    """Sum one contiguous bucket of the flat gradient over ranks, in place, on the caller's
    current stream."""
    dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)


def allreduce_loss(loss3, group=None):
    dist.all_reduce(loss3, op=dist.ReduceOp.SUM, group=group)


def allreduce_err(err, group=None):
    """MAX of the recurrence timeout words over ranks (int32 [1]), before the fused Adam reads
    it: a timeout on any rank leaves that rank's share of the summed gradient undefined, so
    every rank must skip the update together or the replicas' weights diverge."""
    dist.all_reduce(err, op=dist.ReduceOp.MAX, group=group)
    return err


def allreduce_count(count, group=None):
    """Global number of valid frames (int tensor [1])."""
    dist.all_reduce(count, op=dist.ReduceOp.SUM, group=group)
    return count
