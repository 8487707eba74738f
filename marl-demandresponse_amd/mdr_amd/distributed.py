"""Multi-GPU: one process per GPU, houses sharded contiguously, RCCL over xGMI for the exchanges.

The path partitions naturally: every house is independent except for ONE scalar
coupling per tick, the cluster power (and, for the common penalty modes, the cluster penalty
sum/max).  Per tick each rank runs phase 1 on its shard, the tiny per-class ON-count slab is
sum-allreduced with RCCL (exact integer counts, so every rank derives the identical P), then
phase 2.  Scalar drivers (outdoor temperature, solar gain, signal) are replicated: every rank
draws them from the same host RNG stream, so nothing is broadcast.  Messages of the
``neighbours`` ring cross shard edges: ``ring_halo`` exchanges the lo/hi edge houses' message
features (all-gather of 2*5 rows per rank).

The RCCL communicator is created by libmdr_hip (ncclCommInitRank) from a unique id that rank 0
draws and ``torch.distributed`` broadcasts, so the per-tick allreduces are issued from C on the
compute stream (``mdr_rollout_sharded``) without a Python round trip per tick.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


class RcclComm:
    """Collectives of a sharded Environment, over the libmdr_hip RCCL communicator."""

    native = True  # the library's own communicator: C rollout loops may issue the collectives

    def __init__(self):
        import torch.distributed as dist

        if not dist.is_initialized():
            raise RuntimeError("init torch.distributed (backend 'nccl' = RCCL) before RcclComm()")
        self.dist = dist
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
    def attach(self, shard) -> None:
        import torch

        if getattr(shard, "_rccl_ready", False):  # (on the shard: a new shard may reuse a freed id)
            return
        lib = shard.lib
        uid = torch.zeros(128, dtype=torch.uint8)
        if self.rank == 0:
            buf = (C.c_uint8 * 128)()
            L.check(lib.mdr_rccl_unique_id(buf), "mdr_rccl_unique_id")
            uid = torch.tensor(list(bytes(buf)), dtype=torch.uint8)
        dev_uid = uid.to(shard.device)
        self.dist.broadcast(dev_uid, src=0)
        host = bytes(dev_uid.cpu().tolist())
        arr = (C.c_uint8 * 128).from_buffer_copy(host)
        L.check(lib.mdr_rccl_init(shard.ctx, arr, self.world, self.rank), "mdr_rccl_init")
        shard._rccl_ready = True

    def allreduce_counts(self, shard) -> None:
        ptr, n = shard.counts_buffer()
        L.check(shard.lib.mdr_rccl_allreduce(shard.ctx, ptr, n, 0, shard.stream()), "allreduce counts")

    def allreduce_penalty(self, shard) -> None:
        p = C.c_void_p()
        L.check(shard.lib.mdr_penalty_buffer(shard.ctx, C.byref(p)), "mdr_penalty_buffer")
        L.check(shard.lib.mdr_rccl_allreduce(shard.ctx, p.value, 1, 1, shard.stream()), "allreduce pen sum")
        L.check(shard.lib.mdr_rccl_allreduce(shard.ctx, p.value + 8, 1, 2, shard.stream()), "allreduce pen max")

    def allreduce_sum(self, shard, t) -> None:
        """In-place double sum over ranks of a device tensor (interpolation sample values, stats)."""
        L.check(shard.lib.mdr_rccl_allreduce(shard.ctx, L.ptr(t), t.numel(), 1, shard.stream()), "allreduce sum")

    def allreduce_max(self, shard, t) -> None:
        """In-place double max over ranks of a device tensor."""
        L.check(shard.lib.mdr_rccl_allreduce(shard.ctx, L.ptr(t), t.numel(), 2, shard.stream()), "allreduce max")

    def allreduce_min(self, shard, t) -> None:
        """In-place double min over ranks of a device tensor."""
        L.check(shard.lib.mdr_rccl_allreduce(shard.ctx, L.ptr(t), t.numel(), 4, shard.stream()), "allreduce min")

    def allreduce_count32(self, shard, t) -> None:
        """In-place sum over ranks of a 32-bit count tensor (uint32 counts viewed as int32)."""
        L.check(shard.lib.mdr_rccl_allreduce(shard.ctx, L.ptr(t), t.numel(), 3, shard.stream()), "allreduce u32")

    def allgather_bytes(self, shard, t):
        """The ranks' equal-size uint8 device tensors, concatenated in rank order."""
        import torch

        out = torch.empty(self.world * t.numel(), dtype=torch.uint8, device=shard.device)
        L.check(shard.lib.mdr_rccl_allgather(shard.ctx, L.ptr(t), L.ptr(out), t.numel(), shard.stream()),
                "allgather")
        return out

    def rollout(self, shard, ticks, actions, mode, rewards, rew_stride) -> None:
        n = shard.n
        L.check(shard.lib.mdr_rollout_sharded(shard.ctx, len(ticks), ticks.ptr(), L.ptr(actions),
                                              n if actions is not None else 0, mode, L.ptr(rewards),
                                              rew_stride, L.ptr(shard.p_dev), shard.stream()),
                "mdr_rollout_sharded")

    def pipeline(self, shard) -> dict:
        """The sharded rollout pipelines the library uses (mdr_rollout_sharded_mode)."""
        w, t = C.c_int(), C.c_int()
        L.check(shard.lib.mdr_rollout_sharded_mode(shard.ctx, C.byref(w), C.byref(t)), "mdr_rollout_sharded_mode")
        return {"window": "count-ahead (side-stream count + allreduce)" if w.value else "one stream",
                "one_tick": "overlapped (reward one launch later)" if t.value else "serial"}

    def ring_halo(self, shard, spec):
        """Message features of the houses just before / after this shard on the global ring."""
        import torch

        k = spec.n_comm
        lo, hi = k // 2, (k + 1) // 2
        m = shard.lib.mdr_msg_width(C.byref(spec))
        if shard.n < max(lo, hi):
            raise NotImplementedError("shards smaller than the ring half-width")
        mine = torch.empty((hi + lo, m), dtype=torch.float32, device=shard.device)
        shard.halo_pack(spec, mine)
        allh = [torch.empty_like(mine) for _ in range(self.world)]
        self.dist.all_gather(allh, mine)
        prev, nxt = allh[(self.rank - 1) % self.world], allh[(self.rank + 1) % self.world]
        # rows [hi, hi+lo) of a pack = that shard's last lo houses; rows [0, hi) = its first hi
        return torch.cat([prev[hi:hi + lo], nxt[:hi]]).contiguous()

    def allgather_cat(self, shard, t, sizes):
        """The ranks' 1-D device tensors (rank r holds sizes[r] elements) concatenated in rank
        order = global house order (all_gather over rows padded to the largest shard)."""
        import torch

        m = max(sizes)
        buf = t if t.numel() == m else torch.cat([t, t.new_zeros(m - t.numel())])
        parts = [torch.empty_like(buf) for _ in range(self.world)]
        self.dist.all_gather(parts, buf.contiguous())
        return torch.cat([p[:s] for p, s in zip(parts, sizes)])

    def allgather_state(self, shard, st: dict, prm: dict, n: int):
        """Full-cluster host copies of the state/params (dict obs of a sharded env: messages
        reference houses on other shards)."""
        import torch

        out_st, out_prm = {}, {}
        for src, dst, keys in ((st, out_st, ("T", "Tm", "on", "lock", "sso")),
                               (prm, out_prm, ("ua", "ca", "cm", "hm", "target", "cap_idx"))):
            for key in keys:
                a = np.asarray(src[key])
                t = torch.from_numpy(np.ascontiguousarray(a.astype(np.float64))).to(shard.device)
                sizes = [None] * self.world
                self.dist.all_gather_object(sizes, int(t.numel()))
                parts = [torch.empty(s, dtype=torch.float64, device=shard.device) for s in sizes]
                self.dist.all_gather(parts, t)
                full = torch.cat(parts).cpu().numpy()
                dst[key] = full.astype(a.dtype) if a.dtype != np.float64 else full
        return out_st, out_prm


def device_view(ptr: int, n: int, typestr: str, device):
    """Zero-copy torch view of n elements of library-owned device memory."""
    import torch

    class _Arr:
        __slots__ = ("__cuda_array_interface__",)

    a = _Arr()
    a.__cuda_array_interface__ = {"shape": (int(n),), "typestr": typestr, "data": (int(ptr), False),
                                  "version": 2, "strides": None}
    return torch.as_tensor(a, device=device)


class TorchComm(RcclComm):
    """The same exchanges issued through ``torch.distributed`` collectives on zero-copy views of
    the library's count / penalty buffers instead of the library's own RCCL communicator.

    With the 'nccl' backend this is still RCCL (torch's communicator); with 'gloo' it lets
    several ranks share one GPU, which is how the sharded device path is tested on a 1-GPU box.
    Rollouts issue one step per tick from Python (no C loop)."""

    native = False

    def attach(self, shard) -> None:
        pass

    def allreduce_counts(self, shard) -> None:
        ptr, n = shard.counts_buffer()
        self.dist.all_reduce(device_view(ptr, n, "<i8", shard.device))  # counts < 2^63: same bits

    def allreduce_penalty(self, shard) -> None:
        p = C.c_void_p()
        L.check(shard.lib.mdr_penalty_buffer(shard.ctx, C.byref(p)), "mdr_penalty_buffer")
        self.dist.all_reduce(device_view(p.value, 1, "<f8", shard.device))
        self.dist.all_reduce(device_view(p.value + 8, 1, "<f8", shard.device), op=self.dist.ReduceOp.MAX)

    def allreduce_sum(self, shard, t) -> None:
        self.dist.all_reduce(t)

    def allreduce_max(self, shard, t) -> None:
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)

    def allreduce_min(self, shard, t) -> None:
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)

    def allreduce_count32(self, shard, t) -> None:
        self.dist.all_reduce(t)

    def allgather_bytes(self, shard, t):
        import torch

        parts = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t.contiguous())
        return torch.cat(parts)

    def pipeline(self, shard) -> dict:
        return {"mode": "torch.distributed per-step"}

    def ring_halo(self, shard, spec):
        """Point-to-point ring halo, paired exactly as the library's RCCL exchange
        (mdr_capi.hip mdr_actor_rollout_sharded): this shard's last lo houses go to rank r+1 and its
        first hi houses to rank r-1; the halo is [lo rows from r-1 | hi rows from r+1].  Distinct
        tags keep the two directions apart when r-1 == r+1 (world 2).  gloo has no device
        send/recv, so its messages are staged through host memory (one copy each way)."""
        import torch

        k = spec.n_comm
        lo, hi = k // 2, (k + 1) // 2
        m = shard.lib.mdr_msg_width(C.byref(spec))
        if shard.n < max(lo, hi):
            raise NotImplementedError("shards smaller than the ring half-width")
        mine = torch.empty((hi + lo, m), dtype=torch.float32, device=shard.device)
        shard.halo_pack(spec, mine)
        if self.world == 1:  # the local wrap-around (the RCCL path's send/recv to self)
            return torch.cat([mine[hi:hi + lo], mine[:hi]]).contiguous()
        host = self.dist.get_backend() == "gloo" and mine.is_cuda
        src = mine.cpu() if host else mine
        recv = torch.empty((lo + hi, m), dtype=torch.float32, device="cpu" if host else mine.device)
        prev, nxt = (self.rank - 1) % self.world, (self.rank + 1) % self.world
        P2P = self.dist.P2POp
        ops = []
        if lo:
            ops += [P2P(self.dist.isend, src[hi:hi + lo].contiguous(), nxt, tag=1),
                    P2P(self.dist.irecv, recv[:lo], prev, tag=1)]
        if hi:
            ops += [P2P(self.dist.isend, src[:hi].contiguous(), prev, tag=2),
                    P2P(self.dist.irecv, recv[lo:], nxt, tag=2)]
        for r in self.dist.batch_isend_irecv(ops):
            r.wait()
        return recv.to(shard.device) if host else recv

    def rollout(self, shard, ticks, actions, mode, rewards, rew_stride) -> None:
        for t in range(len(ticks)):
            tk = ticks.struct(t)
            a = actions[t] if actions is not None else None
            shard.power_counts(a, mode, tk.tick)
            self.allreduce_counts(shard)
            shard.step(a, mode, tk, reward=rewards[t] if rew_stride else rewards)


class HostComm(TorchComm):
    """The library's sharded C loops (mdr_rollout_begin / mdr_rollout_sharded /
    mdr_actor_rollout_sharded: count-ahead window pipeline, per-tick loops, actor + ring halo)
    with their exchanges handed to ``torch.distributed`` through mdr_comm_host callbacks instead of
    the library's RCCL communicator.  Over gloo several ranks share one GPU, so the C loops run at
    world 3..8 on a 1-GPU box exactly as they run over RCCL, one collective call for one RCCL call
    (the library synchronises the stream first; the callback finishes the exchange before it
    returns).  Python-level exchanges (greedy stages, table obs, dict obs) are TorchComm's."""

    native = True

    def attach(self, shard) -> None:
        if getattr(shard, "_host_comm", None) is self:
            return
        import torch

        dist = self.dist
        gloo = dist.get_backend() == "gloo"
        dev = shard.device
        ops = {0: ("<i8", dist.ReduceOp.SUM), 1: ("<f8", dist.ReduceOp.SUM), 2: ("<f8", dist.ReduceOp.MAX),
               3: ("<u4", dist.ReduceOp.SUM), 4: ("<f8", dist.ReduceOp.MIN)}

        def finish(t, host):
            if host is not None:
                t.copy_(host)
            torch.cuda.synchronize(dev)

        def allreduce(user, buf, count, op):
            try:
                typ, rop = ops[op]
                t = device_view(buf, count, typ if typ != "<u4" else "<i4", dev)
                h = t.cpu() if gloo else None
                dist.all_reduce(h if gloo else t, op=rop)
                finish(t, h)
                return 0
            except Exception as e:  # noqa: BLE001  (an exception must not cross the C frame)
                self.error = e
                return -1

        def sendrecv(user, send, sbytes, dst, recv, rbytes, src, tag):
            try:
                s_t = device_view(send, sbytes, "|u1", dev)
                r_t = device_view(recv, rbytes, "|u1", dev)
                s_h = s_t.cpu() if gloo else s_t
                r_h = torch.empty(rbytes, dtype=torch.uint8) if gloo else r_t
                for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, s_h, dst, tag=tag),
                                                 dist.P2POp(dist.irecv, r_h, src, tag=tag)]):
                    w.wait()
                finish(r_t, r_h if gloo else None)
                return 0
            except Exception as e:  # noqa: BLE001
                self.error = e
                return -1

        self._cbs = (L.HOST_ALLREDUCE_FN(allreduce), L.HOST_SENDRECV_FN(sendrecv))  # (kept alive)
        self.error = None
        L.check(shard.lib.mdr_comm_host(shard.ctx, self.world, self.rank, self._cbs[0], self._cbs[1], None),
                "mdr_comm_host")
        shard._host_comm = self

    def rollout(self, shard, ticks, actions, mode, rewards, rew_stride) -> None:
        RcclComm.rollout(self, shard, ticks, actions, mode, rewards, rew_stride)

    def pipeline(self, shard) -> dict:
        return RcclComm.pipeline(self, shard)


def make_comm(kind: str = "auto"):
    """Communicator for a sharded Environment: 'rccl' (libmdr_hip's own RCCL communicator, per-tick
    allreduces issued from C), 'torch' (torch.distributed collectives), 'host' (the library's C
    loops with torch.distributed collectives as callbacks), or 'auto' (rccl, falling
    back to torch with a warning if the library communicator cannot be created)."""
    if kind == "torch":
        return TorchComm()
    if kind == "host":
        return HostComm()
    if kind == "rccl":
        return RcclComm()
    if kind != "auto":
        raise ValueError(f"unknown comm kind {kind!r}")
    return _AutoComm()


class _AutoComm(RcclComm):
    def attach(self, shard) -> None:
        try:
            super().attach(shard)
        except Exception as e:  # noqa: BLE001
            import warnings

            warnings.warn(f"libmdr RCCL communicator unavailable ({e}); using torch.distributed collectives")
            self.__class__ = TorchComm
