"""Multi-GPU orchestration: one process per GPU, one global particle filter.

Every rank holds a contiguous, chunk-aligned shard of the particles (eslam_gpu_set_comm,
include/eslam_gpu.h).  The library calls back into this module at the three exchange
points of an update (SURVEY.md 8e -- the reference has one CPU filter, no distribution):

  allgather   the ~0.5 KB exact statistics record of each rank, the 8-byte fixed-point
              weight totals, the per-destination send counts
  alltoallv   the particles whose stratified draws land in another rank's slice

``TorchComm`` implements both with torch.distributed: RCCL over xGMI on device buffers
(backend "nccl", device_memory=1, the collectives are queued on the context's HIP stream)
or gloo on host buffers (device_memory=0; the library stages through pinned memory) --
the CPU tests run the oracle's sharded mode through the same callbacks.

``RcclShardedGpuFilter`` skips the host language altogether: the library joins an RCCL
communicator itself (eslam_gpu_set_comm_rccl) and issues ncclAllGather / grouped
ncclSend+ncclRecv on the context's stream; torch.distributed only broadcasts the 128-byte
RCCL id once.  No callback and no cross-stream hand-off sits on the step's critical path.
"""
import ctypes as C

import numpy as np

import eslam_abi as A


def _host_u8(ptr, nbytes):
    import torch
    if nbytes == 0:
        return torch.empty(0, dtype=torch.uint8)
    buf = (C.c_uint8 * nbytes).from_address(ptr)
    return torch.from_numpy(np.ctypeslib.as_array(buf))


class _DevBuf:
    """A raw device pointer seen by torch through __cuda_array_interface__."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3, "strides": None}


def _dev_u8(ptr, nbytes, device):
    import torch
    if nbytes == 0:
        return torch.empty(0, dtype=torch.uint8, device=device)
    return torch.as_tensor(_DevBuf(ptr, nbytes), device=device)


class TorchComm:
    """eslam_comm over an initialised torch.distributed process group."""

    def __init__(self, group=None, device_memory=None, device=None):
        import torch
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.nranks = dist.get_world_size(group)
        if self.nranks > A.MAX_RANKS:
            raise ValueError(f"at most {A.MAX_RANKS} ranks")
        backend = dist.get_backend(group)
        if device_memory is None:
            device_memory = backend == "nccl"
        self.device_memory = bool(device_memory)
        self.device = device if device is not None else (torch.cuda.current_device() if self.device_memory else None)
        self.error = None
        self._ag = A.ALLGATHER_FN(self._allgather)
        self._a2a = A.ALLTOALLV_FN(self._alltoallv)
        self.struct = A.Comm(None, self.rank, self.nranks, 1 if self.device_memory else 0, 0, self._ag, self._a2a)

    # -- callbacks (errors are kept and reported as a nonzero return: the C side raises) --
    def _stream_ctx(self, stream):
        import contextlib
        import torch
        if not self.device_memory or not stream:
            return contextlib.nullcontext()
        return torch.cuda.stream(torch.cuda.ExternalStream(stream, device=self.device))

    def _allgather(self, user, send, recv, nbytes, stream):
        try:
            with self._stream_ctx(stream):
                if self.device_memory:
                    src = _dev_u8(send, nbytes, self.device)
                    dst = _dev_u8(recv, nbytes * self.nranks, self.device)
                    self.dist.all_gather_into_tensor(dst, src, group=self.group)
                else:
                    src = _host_u8(send, nbytes)
                    dst = _host_u8(recv, nbytes * self.nranks)
                    outs = list(dst.split(nbytes)) if nbytes else [dst] * self.nranks
                    self.dist.all_gather(outs, src, group=self.group)
            return 0
        except Exception as e:          # noqa: BLE001 -- reported through the C return code
            self.error = e
            return 1

    def _alltoallv(self, user, send, send_bytes, recv, recv_bytes, stream):
        try:
            sb = [int(send_bytes[r]) for r in range(self.nranks)]
            rb = [int(recv_bytes[r]) for r in range(self.nranks)]
            with self._stream_ctx(stream):
                if self.device_memory:
                    src = _dev_u8(send, sum(sb), self.device)
                    dst = _dev_u8(recv, sum(rb), self.device)
                else:
                    src = _host_u8(send, sum(sb))
                    dst = _host_u8(recv, sum(rb))
                self.dist.all_to_all_single(dst, src, output_split_sizes=rb, input_split_sizes=sb, group=self.group)
            return 0
        except Exception as e:          # noqa: BLE001
            self.error = e
            return 1


class ShardedGpuFilter:
    """The GPU filter of one rank of an n_global-particle filter sharded over the group."""

    def __init__(self, cfg, n_global, comm, device=0):
        import eslam_amd
        self.comm = comm
        self.bounds = A.shard_bounds(n_global, comm.nranks, cfg.sum_chunk_rows)
        cfg.particle_count = n_global
        self.f = eslam_amd.GpuFilter(cfg, device=device)
        if comm.device_memory:
            import torch
            # the context queues on torch's current stream: the RCCL collectives order
            # against it without host synchronisation
            self.f._check(self.f.L.eslam_gpu_set_stream(self.f.h, C.c_void_p(torch.cuda.current_stream().cuda_stream)))
        gb = (C.c_uint64 * len(self.bounds))(*self.bounds)
        self._gb = gb
        self.f._check(self.f.L.eslam_gpu_set_comm(self.f.h, C.byref(comm.struct), n_global, gb))
        self.n_global = n_global
        self.gbase = self.bounds[comm.rank]
        self.n_local = self.bounds[comm.rank + 1] - self.gbase

    def __getattr__(self, name):
        return getattr(self.f, name)

    def close(self):
        """Collective: every rank completes the exchange it may still owe, then frees its context."""
        if getattr(self.f, "h", None):
            self.f.finish()
        self.f.close()


class RcclShardedGpuFilter:
    """ShardedGpuFilter whose exchanges the library drives over its own RCCL communicator.
    Collective: every rank of the torch.distributed group constructs it together."""

    def __init__(self, cfg, n_global, rank, nranks, device=0, group=None):
        import torch
        import torch.distributed as dist
        import eslam_amd
        L = eslam_amd.load_library()
        self.bounds = A.shard_bounds(n_global, nranks, cfg.sum_chunk_rows)
        cfg.particle_count = n_global
        self.f = eslam_amd.GpuFilter(cfg, device=device)
        uid = (C.c_uint8 * 128)()
        if rank == 0:
            self.f._check(L.eslam_gpu_rccl_unique_id(uid))
        # one broadcast of the id (device tensor: the nccl backend moves CUDA tensors)
        t = torch.tensor(list(bytes(uid)), dtype=torch.uint8,
                         device=f"cuda:{device}" if dist.get_backend(group) == "nccl" else "cpu")
        dist.broadcast(t, src=0, group=group)
        uid = (C.c_uint8 * 128)(*t.cpu().tolist())
        gb = (C.c_uint64 * len(self.bounds))(*self.bounds)
        self._gb = gb
        self.f._check(L.eslam_gpu_set_comm_rccl(self.f.h, nranks, rank, uid, n_global, gb))
        self.n_global = n_global
        self.gbase = self.bounds[rank]
        self.n_local = self.bounds[rank + 1] - self.gbase

    def __getattr__(self, name):
        return getattr(self.f, name)

    def close(self):
        """Collective: every rank completes the exchange it may still owe, then frees its context."""
        if getattr(self.f, "h", None):
            self.f.finish()
        self.f.close()
