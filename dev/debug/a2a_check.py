"""all_to_all_single correctness vs message size on the real backend (torchrun)."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


CHUNKED = "--chunked" in sys.argv


def main():
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    dev = int(os.environ.get("LOCAL_RANK", 0)) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    bad = 0
    for mb in (64, 256, 512, 768, 1024, 1536, 2560):
        n = mb << 20
        n -= n % (world * 160)
        x = (torch.arange(n, device="cuda", dtype=torch.int64) * 2654435761 + rank).to(torch.uint8)
        y = torch.empty_like(x)
        if CHUNKED:
            from libsplinter_amd.parallel.sharded import _Coll
            _Coll(None).all_to_all(y, x)
        else:
            dist.all_to_all_single(y, x)
        torch.cuda.synchronize()
        if CHUNKED and world == 1:  # the uneven-split (_route) form through the same chunking
            y2 = torch.empty_like(x)
            _Coll(None).all_to_all(y2, x, [n], [n])
            torch.cuda.synchronize()
            nb = int((y2 != x).sum())
            print(f"chunked-uneven {mb} MiB: mismatching bytes {nb}", flush=True)
            bad += nb
            del y2
        # world == 1: y must equal x
        ref = x if world == 1 else None
        if ref is not None:
            diff = (y != ref)
            nbad = int(diff.sum())
            first = int(torch.nonzero(diff)[0].item()) if nbad else -1
            print(f"{'chunked' if CHUNKED else 'single'} {mb} MiB: mismatching bytes {nbad}, first at {first}", flush=True)
            bad += nbad
        del x, y
    dist.destroy_process_group()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
