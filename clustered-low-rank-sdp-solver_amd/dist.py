"""Multi-GPU plumbing: one process per GPU, the library's cross-rank exchange over
torch.distributed (backend "nccl" = RCCL over xGMI on ROCm; "gloo" for CPU-side tests).

The library (include/clrsdp.h) calls the registered exchange in the middle of a stage with its
work enqueued on its own stream; the collective is issued on that same stream (wrapped as a
torch ExternalStream), so an RCCL all-gather is ordered after the partials were written and
before their rank-ordered reduction, with no host synchronisation.  Payloads are the few cross-cluster quantities of one iteration (Q:
n_y^2 words, three n_y-vectors, ~10 scalars), so the exchange is latency-bound.
"""
from __future__ import annotations

import os


class TorchExchange:
    def __init__(self, local_rank: int, backend: str = None, device: str = "cuda"):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        backend = backend or os.environ.get("CLRSDP_EXCHANGE_BACKEND", "nccl")
        self.backend = backend
        if device == "cuda":
            torch.cuda.set_device(local_rank)
        if not dist.is_initialized():
            if backend == "nccl":
                try:
                    dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
                except Exception as e:  # keep the run alive: host-staged gloo exchange instead
                    print(f"[clrsdp] RCCL process group failed ({e!r}); falling back to gloo",
                          flush=True)
                    self.backend = "gloo"
                    dist.init_process_group("gloo")
            else:
                dist.init_process_group(backend)
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.local_rank = local_rank
        self.dev = None

    def attach(self, dev):
        torch = self.torch
        nbytes = dev.exchange_bytes()
        self.send = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
        self.recv = torch.zeros(nbytes * self.world, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        self.stream = torch.cuda.ExternalStream(dev.stream_ptr())
        dev.set_exchange(self._exchange, self.send.data_ptr(), self.recv.data_ptr())
        self.dev = dev

    def _exchange(self, ctx, tag, nbytes, stream):
        try:
            w = self.world
            torch = self.torch
            with torch.cuda.stream(self.stream):
                if self.backend == "nccl":
                    self.dist.all_gather_into_tensor(self.recv[:nbytes * w], self.send[:nbytes])
                else:  # host staging for gloo (tests on a single GPU)
                    self.stream.synchronize()
                    src = self.send[:nbytes].cpu()
                    outs = [torch.empty_like(src) for _ in range(w)]
                    self.dist.all_gather(outs, src)
                    self.recv[:nbytes * w].copy_(torch.cat(outs).to("cuda"))
                    self.stream.synchronize()
            return 0
        except Exception as e:  # never let an exception cross the C ABI
            print(f"[clrsdp exchange tag {tag}] {e!r}", flush=True)
            return 1

    def barrier(self):
        if self.backend == "nccl":
            self.dist.barrier(device_ids=[self.local_rank])
        else:
            self.dist.barrier()

    def max_over_ranks(self, v: float) -> float:
        torch = self.torch
        dev = "cuda" if self.backend == "nccl" else "cpu"
        t = torch.tensor([float(v)], dtype=torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist.is_initialized():
            self.dist.destroy_process_group()
