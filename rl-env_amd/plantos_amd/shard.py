"""Env sharding across the GPUs of one node.

Envs are independent, so a job of W ranks x n envs is W disjoint shards: rank r
owns global env ids [r*n, (r+1)*n) (``env_id_offset = r*n``: the device-rng map
stream is keyed by the GLOBAL id, so a sharded job reproduces the single-GPU
batch bit for bit).  Nothing is exchanged during a step.  The only collective is
at the host boundary, when one consumer (a policy on rank 0) needs the global
batch: ``gather_outputs`` moves (obs, reward, terminated, truncated) to the root
(RCCL ``gather`` over xGMI on GPUs; gloo on CPU in the tests) and
``scatter_actions`` hands the root's actions back to the shards.
"""
import torch
import torch.distributed as dist


def shard_range(rank, world, envs_per_rank):
    """Global env ids of one rank's shard."""
    return rank * envs_per_rank, (rank + 1) * envs_per_rank


class ShardedPlantOS:
    """One rank's shard plus the host-boundary collectives.

    ``batch_factory(n, env_id_offset=..., seed=...)`` builds the local batch
    (PlantOSBatch on the rank's GPU by default).
    """

    def __init__(self, envs_per_rank, seed=0, batch_factory=None, group=None, **cfg):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.n = int(envs_per_rank)
        lo, _ = shard_range(self.rank, self.world, self.n)
        if batch_factory is None:
            from .batch import PlantOSBatch
            dev = torch.device("cuda", torch.cuda.current_device())
            batch_factory = lambda n, **kw: PlantOSBatch(n, device=dev, **cfg, **kw)  # noqa: E731
        self.batch = batch_factory(self.n, env_id_offset=lo, seed=seed)
        self._gbuf = None

    @property
    def device(self):
        return self.batch.device

    def step(self, actions_local):
        return self.batch.step(actions_local)

    def _root_bufs(self, obs, rew, te, tr):
        if self._gbuf is None:
            mk = lambda t: [torch.empty_like(t) for _ in range(self.world)]  # noqa: E731
            self._gbuf = (mk(obs), mk(rew), mk(te), mk(tr))
        return self._gbuf

    def gather_outputs(self, root=0):
        """(obs, reward, terminated, truncated) of all ranks, concatenated in global
        env order on `root` (None elsewhere)."""
        b = self.batch
        outs = (b.obs, b.reward, b.terminated, b.truncated)
        if self.world == 1:
            return outs
        bufs = self._root_bufs(*outs) if self.rank == root else (None, None, None, None)
        for t, lst in zip(outs, bufs):
            dist.gather(t, lst, dst=root, group=self.group)
        if self.rank != root:
            return None
        return tuple(torch.cat(lst, 0) for lst in bufs)

    def scatter_actions(self, actions_global=None, root=0):
        """Root's global action vector -> this rank's shard (int64 [n])."""
        out = torch.empty(self.n, dtype=torch.int64, device=self.device)
        if self.world == 1:
            out.copy_(actions_global.reshape(-1))
            return out
        chunks = None
        if self.rank == root:
            a = actions_global.reshape(-1).to(device=self.device, dtype=torch.int64)
            chunks = list(a.split(self.n))
        dist.scatter(out, chunks, src=root, group=self.group)
        return out

    def close(self):
        self.batch.close()
