"""Env sharding across the GPUs of one node.

Envs are independent, so a job of W ranks x n envs is W disjoint shards: rank r
owns global env ids [r*n, (r+1)*n) (``env_id_offset = r*n``: the device-rng map
stream is keyed by the GLOBAL id, so a sharded job reproduces the single-GPU
batch bit for bit).  Nothing is exchanged during a step.  The only collective is
at the host boundary, when one consumer (a policy on rank 0) needs the global
batch: ``gather_outputs`` moves (obs, reward, terminated, truncated) to the root
as ONE packed buffer per rank (RCCL ``gather`` over xGMI on GPUs; gloo on CPU in
the tests; ``step_gather`` pipelines it behind the next step) and
``scatter_actions`` hands the root's actions back to the shards.

``codes=True`` (the geometries with a byte-coded sector kernel, e.g. BASELINE config
5's 20x20 / 16 rays): every rank's step writes its obs as byte codes (codes.py,
pe_step_codes), so each rank contributes 5C+27 bytes of obs per env instead of
4(5C+27) (7.1 MB instead of 28.4 MB per rank at 65536 envs), and the root expands
all ranks' codes in ONE kernel straight into contiguous f32 [W*n, D] / reward /
terminated / truncated tensors (``unpack``; no concatenation copy).
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

    def __init__(self, envs_per_rank, seed=0, batch_factory=None, group=None, codes=False, **cfg):
        if "obs_codes" in cfg:
            raise TypeError("ShardedPlantOS: pass codes=True, not obs_codes (the shard's unpack follows `codes`)")
        self.group = group
        self.codes = bool(codes)
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # the collectives run whenever a process group exists -- also with one rank (a
        # torchrun job of one: the same RCCL code path, gathering to itself)
        self._coll = dist.is_initialized()
        self.n = int(envs_per_rank)
        lo, _ = shard_range(self.rank, self.world, self.n)
        if batch_factory is None:
            from .batch import PlantOSBatch
            dev = torch.device("cuda", torch.cuda.current_device())
            batch_factory = lambda n, **kw: PlantOSBatch(n, device=dev, **cfg, **kw)  # noqa: E731
        extra = {"obs_codes": True} if self.codes else {}
        self.batch = batch_factory(self.n, env_id_offset=lo, seed=seed, **extra)
        # the io layout the batch actually writes (a factory may set it regardless of `codes`)
        self.codes = bool(getattr(self.batch, "obs_codes", False))
        self._slots = None
        self._last_io = None  # the buffer the latest step wrote (None: the batch's own io)
        self._gbuf = None     # root: gather_outputs' [W, io_bytes] buffer

    @property
    def device(self):
        return self.batch.device

    def step(self, actions_local):
        self._last_io = None
        return self.batch.step(actions_local)

    def io_bytes(self):
        """Bytes of one rank's packed step outputs (what one gather moves per rank)."""
        return self.batch.io_bytes()

    def _gather_buffer(self):
        """Root: one contiguous [W, io_bytes] buffer the W ranks' buffers are gathered
        into (its rows are the gather list: no copy to assemble it afterwards)."""
        return torch.empty((self.world, self.io_bytes()), dtype=torch.uint8, device=self.device)

    def _pack(self):
        """The latest step's outputs of this shard as ONE flat u8 buffer: the buffer
        that step wrote (the batch's io, or step_gather's slot) -- no copy."""
        if self._last_io is not None:
            return self._last_io
        io = getattr(self.batch, "io", None)
        if io is not None:
            return io
        b = self.batch
        return torch.cat([t.contiguous().view(-1).view(torch.uint8)
                          for t in (b.obs, b.reward, b.terminated, b.truncated)])

    def unpack(self, flats, out=None):
        """The W ranks' packed buffers (rank order: ``gathered(slot)``'s [W, io_bytes]
        rows) as the global (obs f32 [W*n, D], reward f32 [W*n], terminated u8,
        truncated u8).  codes: ONE expansion kernel writes them into fresh tensors, or
        into `out` (four contiguous tensors the caller owns and may reuse: an explicit
        opt-in, so that both modes hand out tensors the next unpack never overwrites);
        otherwise the f32 parts are concatenated."""
        n = self.n
        D = self.batch.obs_dim
        if self.codes:
            src = flats if isinstance(flats, torch.Tensor) else torch.stack(list(flats))
            W = src.shape[0] if src.dim() == 2 else 1
            if out is None:
                out = self.new_outputs(W)
            self.batch.expand_codes(src.reshape(-1), W, *out)
            return out
        sizes = (4 * n * D, 4 * n, n, n)
        parts = [[], [], [], []]
        for f in flats:
            off = 0
            for k, sz in enumerate(sizes):
                parts[k].append(f[off:off + sz])
                off += sz
        obs = torch.cat(parts[0]).view(torch.float32).view(-1, D)
        return obs, torch.cat(parts[1]).view(torch.float32), torch.cat(parts[2]), torch.cat(parts[3])

    def new_outputs(self, W=None):
        """Four contiguous tensors for the expanded global outputs of W ranks (default:
        this job's world): obs f32 [W*n, D], reward f32, terminated u8, truncated u8 --
        the `out` a consumer that reuses its buffers passes to unpack."""
        W = self.world if W is None else int(W)
        n, D, dev = self.n, self.batch.obs_dim, self.device
        return (torch.empty((W * n, D), dtype=torch.float32, device=dev), torch.empty(W * n, dtype=torch.float32, device=dev),
                torch.empty(W * n, dtype=torch.uint8, device=dev), torch.empty(W * n, dtype=torch.uint8, device=dev))

    def gather_outputs(self, root=0):
        """(obs, reward, terminated, truncated) of all ranks, concatenated in global
        env order on `root` (None elsewhere): ONE gather of each rank's packed
        output buffer (RCCL over xGMI on GPUs)."""
        flat = self._pack()
        if not self._coll:
            return self.unpack(flat.view(1, -1))
        lst = None
        if self.rank == root:
            if self._gbuf is None:
                self._gbuf = self._gather_buffer()
            lst = list(self._gbuf)
        dist.gather(flat, lst, dst=root, group=self.group)
        if self.rank != root:
            return None
        return self.unpack(self._gbuf)

    def step_gather(self, actions_local, root=0):
        """Pipelined step + host-boundary gather (GPU batches): the step writes into
        one of two output buffers and its gather to `root` is issued asynchronously,
        so the gather of step t overlaps step t+1; before a buffer is written again
        the stream waits for its previous gather.  Returns the slot used; the
        gathered buffers of a slot are `gathered(slot)` on root once `flush()` (or
        the slot's next use) has waited for it; `unpack(gathered(slot))` gives the
        global (obs, reward, terminated, truncated).  With one rank nothing is
        gathered: `gathered(slot)` is the slot itself."""
        b = self.batch
        if self._slots is None:
            self._slots = [b.new_io(), b.new_io()]
            self._glist = [self._gather_buffer() if (self.rank == root and self._coll) else None for k in range(2)]
            self._work = [None, None]
            self._root = root
            self._k = 0
        k = self._k
        self._k ^= 1
        if self._work[k] is not None:
            self._work[k].wait()  # the stream waits for the slot's previous gather
            self._work[k] = None
        b.step(actions_local, io=self._slots[k])
        self._last_io = self._slots[k]
        if self._coll:
            lst = list(self._glist[k]) if self._glist[k] is not None else None
            self._work[k] = dist.gather(self._slots[k], lst, dst=root, group=self.group, async_op=True)
        return k

    def gathered(self, k):
        """Root: the W ranks' packed buffers of slot k as the rows of one [W, io_bytes]
        tensor (rank order); None elsewhere.  Without a process group: slot k itself
        as a [1, io_bytes] view."""
        if self._slots is None:
            raise ValueError("no step_gather yet")
        if not self._coll:
            return self._slots[k].view(1, -1)
        return self._glist[k]

    def wait(self, k):
        """Wait for slot k's gather only (the other slot's may stay in flight)."""
        if self._slots is not None and self._work[k] is not None:
            self._work[k].wait()
            self._work[k] = None

    def flush(self):
        if self._slots is None:
            return
        for k in range(2):
            self.wait(k)

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
