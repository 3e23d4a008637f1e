"""xGMI peer-to-peer all-reduce for tensor-parallel activations (``csrc/p2p.hip``).

SURVEY §2.3 / §5.8: TP makes 4 all-reduces of the fp32 residual ``[tokens, d_model]`` per
layer (+1 for the head).  On an 8×MI355X node every GPU has a direct xGMI link to every other
one; a ring all-reduce drives one outgoing link per step, while this two-shot kernel lets every
rank read its slice from all peers at once (reduce-scatter), then read every peer's reduced
slice (all-gather), through IPC-mapped peer buffers.

Being ordinary stream-ordered kernels (barriers are device-side epoch flags), the collective is
captured INTO the step's hipGraph: the TP step no longer cuts its graph at every all-reduce the
way an eager RCCL call does.  The sum runs in rank order on every rank, so TP replicas stay
bitwise identical.  RCCL remains the path for anything else (scalars, non-fp32, oversize).

Handles are exchanged once over the process group (``all_gather_object``), so the same code runs
on a real node (RCCL group) and in the one-GPU multi-process tests (gloo group, all ranks on one
device — IPC within a device works the same way).

Small messages (the vocab-parallel CE row statistics and label logits, the grad-norm scalar) take a
one-shot variant (one barrier; every rank sums all peers' buffers itself), so a TP step issues no
RCCL call at all: :class:`parallel.tp.TPComm` gathers by summing zero-padded slots.
"""

from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from ..ops import _native as N


def _pci_bus_id(L, dev: int) -> str:
    buf = ctypes.create_string_buffer(64)
    N.check(L.dtc_device_pci_bus_id(dev, buf, 64), "hipDeviceGetPCIBusId")
    return buf.value.decode().lower()


def check_peer_access(L, rank: int, dev: int, peers) -> dict:
    """``peers``: [(rank, pci bus id)] of the group.  Every peer GPU must be reachable by direct
    loads from this one (hipDeviceCanAccessPeer over xGMI); raises naming the rank and peer
    otherwise — the P2P all-reduce never silently switches paths.  Peers on this same GPU (the
    one-GPU multi-process tests) need no peer access.  Returns {peer rank: "self" | "xgmi" |
    "not-visible"} (a peer GPU outside this process's visible set cannot be queried; its IPC
    mapping below still has to succeed)."""
    mine = _pci_bus_id(L, dev)
    n = ctypes.c_int(0)
    N.check(L.dtc_device_count(ctypes.byref(n)), "hipGetDeviceCount")
    ordinal = {_pci_bus_id(L, d): d for d in range(n.value)}
    out = {}
    for p, bus in peers:
        if p == rank:
            continue
        if bus == mine:
            out[p] = "self"
            continue
        if bus not in ordinal:
            out[p] = "not-visible"
            continue
        ok = ctypes.c_int(0)
        N.check(L.dtc_can_access_peer(dev, ordinal[bus], ctypes.byref(ok)), "hipDeviceCanAccessPeer")
        if not ok.value:
            raise RuntimeError(f"P2P all-reduce: rank {rank} (GPU {dev}, {mine}) cannot access rank {p}'s GPU "
                               f"({bus}) directly; use tp_comm: rccl")
        out[p] = "xgmi"
    return out


class P2PAllReduce:
    def __init__(self, group, rank: int, world: int, device, max_bytes: int):
        assert 1 <= world <= 8, "P2P all-reduce supports up to 8 ranks (one xGMI hive)"
        self.rank, self.world = rank, world
        self.device = torch.device(device)
        self.half = (int(max_bytes) + 4095) // 4096 * 4096
        L = N.lib()
        total = int(L.dtc_p2p_flag_bytes()) + 2 * self.half
        ptr = ctypes.c_void_p()
        handle = ctypes.create_string_buffer(64)
        with torch.cuda.device(self.device):
            N.check(L.dtc_p2p_alloc(total, ctypes.addressof(ptr), ctypes.addressof(handle)), "dtc_p2p_alloc")
        self._own = ptr.value
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        info = [None] * world
        dist.all_gather_object(info, (bytes(handle.raw), _pci_bus_id(L, dev)), group=group)
        self.peer_paths = check_peer_access(L, rank, dev, [(p, bus) for p, (_, bus) in enumerate(info)])
        bases = []
        self._opened = []
        with torch.cuda.device(self.device):
            for p, (h, bus) in enumerate(info):
                if p == rank:
                    bases.append(self._own)
                    continue
                q = ctypes.c_void_p()
                hb = ctypes.create_string_buffer(h, 64)
                rc = L.dtc_p2p_open(ctypes.addressof(hb), ctypes.addressof(q))
                if rc != 0:
                    raise RuntimeError(f"P2P all-reduce: rank {rank} could not map rank {p}'s buffer (GPU {bus}): "
                                       f"hipIpcOpenMemHandle error {rc}")
                bases.append(q.value)
                self._opened.append(q.value)
        self._bases = (ctypes.c_void_p * 8)(*(bases + [None] * (8 - world)))
        self._bases_ptr = ctypes.addressof(self._bases)
        self.epoch = torch.zeros(1, dtype=torch.int32, device=self.device)
        # calls issued so far (host mirror of epoch / 2): the buffer half of the next call is calls & 1
        self.calls = 0
        self._flag_bytes = int(L.dtc_p2p_flag_bytes())
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        # all ranks' flag areas are zero before anyone's first barrier can run
        torch.cuda.synchronize(self.device)
        dist.barrier(group=group)

    def supports(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() % 4 == 0
                and t.numel() * 4 <= self.half)

    def all_reduce_(self, t: torch.Tensor, mode: int = 0) -> torch.Tensor:
        """In-place sum over the group.  mode 0: one-shot (one barrier, every rank reads every peer) at
        W = 2 and for small messages (<= 1 MB at W <= 4, 512 KB at W = 8), else two-shot (reduce-scatter
        + all-gather, 2 (W-1)/W of the bytes per rank); 1 / 2 force two-shot / one-shot."""
        N.check(N.lib().dtc_p2p_allreduce(t.data_ptr(), t.data_ptr(), t.numel(), self._bases_ptr, self.rank, self.world,
                                          self.half, self.epoch.data_ptr(), self.err.data_ptr(), int(mode),
                                          N.stream_ptr(t.device)), "dtc_p2p_allreduce")
        self.calls += 1
        return t

    def staged_out(self, numel: int, dtype=torch.bfloat16):
        """Where the producer of the NEXT call's bf16 payload should write it (this rank's buffer half
        of that call, a :class:`ops.gemm.RawOut`), or None if it does not fit.  The next call must then
        be :meth:`all_reduce_bf16` with ``x=None``.  The half is ``calls & 1``; :meth:`end_step` keeps
        the calls per step even so the half of each call site is the same on every graph replay."""
        from ..ops.gemm import RawOut

        esz = 2 if dtype == torch.bfloat16 else (4 if dtype == torch.float32 else 0)
        if not esz or numel % 8 or numel * esz > self.half:
            return None
        return RawOut(self._own + self._flag_bytes + (self.calls & 1) * self.half, dtype, self.device)

    def end_step(self):
        """Pad the step's calls to an even count with a payload-free barrier round (epoch + 2)."""
        if self.calls & 1:
            N.check(N.lib().dtc_p2p_barrier_round(self._bases_ptr, self.rank, self.world, self.epoch.data_ptr(),
                                                  self.err.data_ptr(), N.stream_ptr(self.device)),
                    "dtc_p2p_barrier_round")
            self.calls += 1

    def supports_bf16(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.numel() % 8 == 0
                and x.numel() * 2 <= self.half)

    def all_reduce_bf16(self, x, out: torch.Tensor, resid=None, bias=None, mode: int = 0) -> torch.Tensor:
        """out (fp32) = resid + bias + Σ_ranks x, x bf16 (the payload), fp32 sums in rank order; ``bias``
        indexed by the last dimension of ``out``.  Same barrier / buffer-half protocol as all_reduce_.
        ``x=None``: the payload (``out.numel()`` values) was written by its producer straight into
        :meth:`staged_out`, so no stage copy runs."""
        ncols = out.shape[-1] if bias is not None else 0
        n = out.numel() if x is None else x.numel()
        assert x is not None or n * 2 <= self.half
        N.check(N.lib().dtc_p2p_allreduce_bf16(N.ptr(x), out.data_ptr(), n, self._bases_ptr, self.rank,
                                               self.world, self.half, self.epoch.data_ptr(), self.err.data_ptr(),
                                               int(mode), N.ptr(resid), N.ptr(bias), ncols, N.stream_ptr(out.device)),
                "dtc_p2p_allreduce_bf16")
        self.calls += 1
        return out

    # ---- sequence parallelism: row-sharded residual stream (parallel/tp.py TPComm.*_rows)
    def supports_rs(self, rows: int, cols: int, dtype) -> bool:
        esz = 2 if dtype == torch.bfloat16 else (4 if dtype == torch.float32 else 0)
        loc = rows // self.world * cols
        return bool(esz) and rows % self.world == 0 and loc % 8 == 0 and rows * cols * esz <= self.half

    def reduce_scatter(self, x, rows: int, cols: int, dtype, out: torch.Tensor, resid=None, bias=None) -> torch.Tensor:
        """out (fp32 [rows / W, cols], this rank's rows) = resid + bias + Σ_ranks x[own rows]; ``x`` the full
        [rows, cols] partial (bf16 / fp32) or None when its producer wrote it into :meth:`staged_out`."""
        n_loc = rows // self.world * cols
        N.check(N.lib().dtc_p2p_reduce_scatter(N.ptr(x), int(dtype == torch.bfloat16), out.data_ptr(), n_loc,
                                               self._bases_ptr, self.rank, self.world, self.half,
                                               self.epoch.data_ptr(), self.err.data_ptr(), N.ptr(resid), N.ptr(bias),
                                               cols if bias is not None else 0, N.stream_ptr(out.device)),
                "dtc_p2p_reduce_scatter")
        self.calls += 1
        return out

    def supports_ag(self, x: torch.Tensor) -> bool:
        nb = x.numel() * x.element_size()
        return x.is_cuda and x.is_contiguous() and nb % 16 == 0 and nb * self.world <= self.half

    def all_gather(self, x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """out [W * rows, ...] (rank-major) = every rank's ``x`` (any dtype, 16-byte multiple)."""
        N.check(N.lib().dtc_p2p_all_gather(x.data_ptr(), out.data_ptr(), x.numel() * x.element_size(),
                                           self._bases_ptr, self.rank, self.world, self.half, self.epoch.data_ptr(),
                                           self.err.data_ptr(), N.stream_ptr(out.device)), "dtc_p2p_all_gather")
        self.calls += 1
        return out

    def check(self):
        """Raise if a barrier timed out (a peer never arrived); call at a host sync point.

        Also checks the buffer-half invariant :meth:`staged_out` relies on: every call advances the
        device epoch by 2, replays included, while the host counter only sees calls issued from Python
        (eager or captured), so the device half ``(epoch >> 1) & 1`` must equal the host half ``calls & 1``
        (true as long as every captured step is padded to an even count by :meth:`end_step`).  A P2P call
        outside the step (eval, a debug all-reduce) without its own :meth:`end_step` flips it, after which
        graph replays would reduce the stale half: raise instead."""
        e = int(self.err.item())
        if e:
            raise RuntimeError(f"P2P all-reduce: rank {self.rank} timed out waiting for rank {e - 1000}")
        dev_half = (int(self.epoch.item()) >> 1) & 1
        if dev_half != (self.calls & 1):
            raise RuntimeError(f"P2P all-reduce: rank {self.rank} buffer-half mismatch (device epoch "
                               f"{int(self.epoch.item())}, host calls {self.calls}): a P2P call outside the step "
                               "left an odd call count; call end_step() after out-of-step P2P use")

    def close(self):
        L = N.lib()
        for q in self._opened:
            L.dtc_p2p_close(ctypes.c_void_p(q))
        self._opened = []
        if self._own:
            L.dtc_p2p_free(ctypes.c_void_p(self._own))
            self._own = None
