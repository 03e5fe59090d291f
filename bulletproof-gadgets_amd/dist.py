"""Multi-GPU plumbing over torch.distributed (RCCL on ROCm; gloo for the CPU
tests), one process per GPU.

Three uses:
* throughput: independent proofs per rank, no data-path collective; the
  bench's barrier and max-over-ranks wall time (`max_over_ranks`);
* one proof sharded across GPUs (`sharded_prove`): the cyclic lane layout
  keeps every commitment MSM and the first lg(N/world) IPP rounds
  rank-local; the partial points/scalars of each step are all-gathered
  (lg N + 3 small collectives per proof) and summed on every rank;
* one big verification sharded across GPUs: each rank sums its slice of the
  verifier's mega-MSM (`bpg_r1cs_verify_shard`), the 32-byte partials are
  all-gathered (RCCL has no elliptic-curve reduction op, so a Ristretto point
  sum cannot be an ncclSum) and every rank adds them on the host
  (`bpg_point_sum`): valid iff the sum is the identity. The exchange is
  world x 33 bytes — latency-bound, a single collective.
"""
import torch
import torch.distributed as dist

IDENTITY = b"\0" * 32


def comm_device():
    """Tensors for collectives live on the rank's GPU under RCCL, on the CPU
    under gloo."""
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_gather_bytes(payload):
    """Every rank contributes `payload` (same length on all ranks); returns
    the list of all ranks' payloads, in rank order."""
    dev = comm_device()
    t = torch.tensor(list(payload), dtype=torch.uint8, device=dev)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [bytes(o.cpu().tolist()) for o in out]


def max_over_ranks(x):
    t = torch.tensor([float(x)], dtype=torch.float64, device=comm_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def combine_verify(bpg, msgs):
    """msgs: per-rank 33-byte messages (ok flag || compressed partial)."""
    if any(m[0] != 1 for m in msgs):
        return False
    return bpg.point_sum([m[1:] for m in msgs]) == IDENTITY


def sharded_prove(ctx, label, view, entropy):
    """Prover::prove (prove.rs:79) of ONE proof split over all ranks of the
    default process group (bpg_r1cs_prove_sharded: rank r holds lanes
    i = j * world + r; partial sums are all-gathered per exchange). Every
    rank returns the same (proof, V)."""
    rank, world = dist.get_rank(), dist.get_world_size()
    if world == 1:
        return ctx.r1cs_prove(label, view, entropy)
    return ctx.r1cs_prove_sharded(label, view, entropy, rank, world, all_gather_bytes)


def sharded_verify_prepared(bpg, prep, label, V, proof, entropy=b"\x05" * 32):
    """The same over a circuit every rank prepared once (ctx.prepare(view,
    verifier=True)): per proof only the transcript replay, the device work of
    this rank's slice and one all-gather of 33 bytes."""
    rank, world = dist.get_rank(), dist.get_world_size()
    if world == 1:
        return prep.verify_one(label, V, proof, entropy)
    ok, part = prep.verify_one(label, V, proof, entropy, rank, world)
    return combine_verify(bpg, all_gather_bytes(bytes([1 if ok else 0]) + part))


def sharded_verify(bpg, ctx, label, view, V, proof, entropy=b"\x05" * 32):
    """Verifier::verify (verify.rs:71) with its mega-MSM split over all ranks
    of the default process group; every rank returns the same verdict."""
    rank, world = dist.get_rank(), dist.get_world_size()
    if world == 1:
        return ctx.r1cs_verify(label, view, V, proof, entropy)
    ok, part = ctx.r1cs_verify_shard(label, view, V, proof, rank, world, entropy)
    return combine_verify(bpg, all_gather_bytes(bytes([1 if ok else 0]) + part))
