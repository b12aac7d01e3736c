"""Data parallelism over RCCL (torch.distributed backend "nccl" == RCCL on ROCm) — SURVEY C48/R01.

One process per GPU (torchrun / MASTER_ADDR env). Each rank computes the gradient of the mean
loss over its local batch into the model's flat fp32 gradient buffer; gradients are summed with
all-reduce and scaled by 1/world (equal local batches => the global-batch mean), then every rank
applies the identical fused SGD update, so replicas stay bit-identical without re-broadcasts.

Overlap: ``BucketedAllReduce`` splits the flat buffer into contiguous buckets at layer
boundaries. Backward produces gradients last-layer-first, so a bucket's all-reduce is issued
(async, on RCCL's stream, ordered after the kernels already queued on the compute stream) as soon
as its lowest layer's wgrad has been launched, overlapping communication with the remaining
backward kernels. Buckets are sized for xGMI ring throughput (a few MB each), not NVSwitch.

CPU runs (tests) use the gloo backend with the same code path.

``RAG_FORCE_PG=1`` initialises the process group even for a single process (WORLD_SIZE = 1, an
RCCL communicator of one rank on a GPU): every collective of the DP path (bucketed gradient
all-reduce in fp32 or bf16, broadcasts, barriers, the search's RootExchange, the watchdog's
c10d store) then runs through the real library on a one-GPU box, where a one-rank all-reduce
must leave every value unchanged.
"""
import datetime
import os
import socket

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def force_pg():
    return os.environ.get("RAG_FORCE_PG", "0") not in ("", "0")


def _single_rank_env():
    """Rendezvous variables for a one-process group (env:// needs them)."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        os.environ["MASTER_PORT"] = str(s.getsockname()[1])
        s.close()
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")


class DPContext(object):
    """One rank of a data-parallel job (one process per GPU, torch.distributed; "nccl" is RCCL
    on ROCm). Enabled when WORLD_SIZE > 1, when RAG_FORCE_PG forces a one-rank group, or, with
    ``adopt=True``, when the process already joined a group (an embedded gloo group, tests):
    a group that merely exists is not adopted by default, and an adopted group
    supplies rank, world AND the local rank (device) together."""

    def __init__(self, device=None, backend=None, timeout_s=600, adopt=False):
        world, rank, local = env_world()
        self.world, self.rank, self.local_rank = world, rank, local
        existing = dist.is_available() and dist.is_initialized()
        self.enabled = world > 1 or force_pg() or (adopt and existing)
        if self.enabled and existing and world == 1:
            # adopted group: the environment says nothing about it
            self.local_rank = local = dist.get_rank() % max(1, torch.cuda.device_count())
        if self.enabled and world == 1 and not existing:
            _single_rank_env()
        if device is None:
            device = torch.device("cuda", local % max(1, torch.cuda.device_count())) \
                if torch.cuda.is_available() else torch.device("cpu")
        self.device = torch.device(device)
        if self.enabled and not dist.is_initialized():
            if self.device.type == "cuda":
                torch.cuda.set_device(self.device)
            # RAG_DIST_BACKEND=gloo: rehearse several ranks on one GPU (RCCL wants one GPU per rank)
            backend = backend or os.environ.get("RAG_DIST_BACKEND") or \
                ("nccl" if self.device.type == "cuda" else "gloo")
            kw = {}
            if backend == "nccl" and self.device.type == "cuda":
                kw["device_id"] = self.device
            dist.init_process_group(backend=backend,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
        self.is_root = self.rank == 0
        self.backend = dist.get_backend() if self.enabled else None
        if self.enabled:
            self.world = dist.get_world_size()
            self.rank = dist.get_rank()
            self.is_root = self.rank == 0

    def broadcast_(self, t, src=0):
        if self.enabled:
            dist.broadcast(t, src)
        return t

    def broadcast_model(self, model):
        """Make every replica start from rank 0's weights."""
        if self.enabled:
            dist.broadcast(model.net.flat, 0)
            model.net.bump()

    def allreduce_mean_(self, t):
        if self.enabled:
            dist.all_reduce(t)
            t.div_(self.world)
        return t

    def allreduce_sum_(self, t):
        if self.enabled:
            dist.all_reduce(t)
        return t

    def barrier(self):
        if self.enabled:
            if self.device.type == "cuda":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def sync_buffers_(self, net):
        """Average the non-trainable running statistics (BatchNorm ``*_running_mean`` /
        ``*_running_std``) of ``net`` over the ranks. They get no gradient, so without this each
        replica would keep its own local-batch averages. The running-mean update is linear in
        the batch mean, so averaging after every step reproduces the global-batch running mean
        exactly (equal local batches); the running variance becomes the mean of the local
        variances."""
        if not self.enabled:
            return
        views = net.buffer_views()
        if not views:
            return
        buf = torch.cat([v.reshape(-1) for v in views])
        dist.all_reduce(buf)
        buf.div_(self.world)
        off = 0
        with torch.no_grad():
            for v in views:
                n = v.numel()
                v.copy_(buf[off:off + n].view_as(v))
                off += n
        net.bump()

    def max_scalar(self, v):
        if not self.enabled:
            return v
        t = torch.tensor([float(v)], device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def shutdown(self):
        if self.enabled and dist.is_initialized():
            dist.destroy_process_group()


class BucketedAllReduce(object):
    """Async all-reduce of a flat gradient buffer in layer-aligned buckets (back to front)."""

    def __init__(self, ctx, flat_grad, layer_offsets, bucket_bytes=4 << 20, timer=None,
                 comm_dtype=None):
        """layer_offsets: ascending start offsets (elements) of each trunk layer's params in
        ``flat_grad``; the tail after the last offset (head params) joins the last bucket.
        ``timer`` (utils.metrics.CommTimer) brackets the exposed wait in ``finish``.
        ``comm_dtype`` (default: env RAG_GRAD_ALLREDUCE_DTYPE, fp32): ``"bf16"`` sends each bucket
        as bf16 (half the xGMI bytes; the sum is rounded to bf16 — every rank receives the same
        values, so replicas stay identical) and widens it back into the fp32 buffer."""
        self.ctx = ctx
        self.flat = flat_grad
        self.timer = timer
        comm_dtype = comm_dtype or os.environ.get("RAG_GRAD_ALLREDUCE_DTYPE", "fp32")
        if comm_dtype not in ("fp32", "bf16"):
            raise ValueError("gradient all-reduce dtype must be fp32 or bf16, got %r"
                             % comm_dtype)
        self.comm = torch.empty(flat_grad.numel(), dtype=torch.bfloat16,
                                device=flat_grad.device) if comm_dtype == "bf16" else None
        self.handles = []
        n = flat_grad.numel()
        # build buckets from the end: [start, end)
        bounds = []
        end = n
        cur_start = n
        for off in reversed(layer_offsets):
            cur_start = off
            if (end - cur_start) * 4 >= bucket_bytes:
                bounds.append((cur_start, end))
                end = cur_start
        if end > 0:
            bounds.append((0, end))
        self.bounds = bounds  # in backward order
        # layer index -> bucket to launch once that layer's grads exist
        self.trigger = {}
        for bi, (s, e) in enumerate(bounds):
            for li, off in enumerate(layer_offsets):
                if off == s:
                    self.trigger[li] = bi
        self._launched = set()

    def reset(self):
        self.handles = []
        self._launched = set()

    def layer_done(self, layer):
        bi = self.trigger.get(layer)
        if bi is None or bi in self._launched or not self.ctx.enabled:
            return
        self._launch(bi)

    def _launch(self, bi):
        s, e = self.bounds[bi]
        buf = self.flat[s:e]
        if self.comm is not None:
            buf = self.comm[s:e]
            buf.copy_(self.flat[s:e])
        self.handles.append(dist.all_reduce(buf, async_op=True))
        self._launched.add(bi)

    def finish(self):
        if not self.ctx.enabled:
            return
        if self.timer is not None:
            self.timer.start()
        for bi in range(len(self.bounds)):
            if bi not in self._launched:
                self._launch(bi)
        for h in self.handles:
            h.wait()
        if self.timer is not None:
            self.timer.stop()
        if self.comm is not None:
            self.flat.copy_(self.comm)
        self.flat.div_(self.ctx.world)
        self.reset()
