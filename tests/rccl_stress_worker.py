"""Worker for tests/test_gpu_xgmi.py: issue()/wait() of the native RcclPlane from two threads.

One thread issues small self send/recv groups back to back while another
polls wait() with a short timeout, queries and releases them -- the pattern
of the data plane's issuer and completer threads.  Run in its own process so
a hang is reported (Python stacks of every thread) instead of stalling the
test session.

    python tests/rccl_stress_worker.py N_GROUPS
"""

from __future__ import annotations

import faulthandler
import os
import queue
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main(n_groups: int) -> None:
    faulthandler.dump_traceback_later(60, exit=True)
    from p2pfl_amd import ops

    C = ops.ext()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    p = C.RcclPlane(C.rccl_unique_id(), 1, 0, 0, 60.0)
    q: "queue.Queue" = queue.Queue()
    errors = []
    progress = {"issued": 0, "done": 0}

    def issuer():
        try:
            for i in range(n_groups):
                a = torch.full((4096,), float(i), device=dev)
                b = torch.empty_like(a)
                gid = p.issue([(0, 0, a), (1, 0, b)], [torch.cuda.current_stream(dev).cuda_stream], 30.0)
                progress["issued"] += 1
                q.put((gid, i, b))
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
        q.put(None)

    def completer():
        try:
            while True:
                item = q.get()
                if item is None:
                    return
                gid, i, b = item
                while p.wait(gid, 0.0005) == 0:
                    p.query(gid)
                p.release(gid)
                if float(b[0]) != float(i) or float(b[-1]) != float(i):
                    errors.append(f"group {i}: wrong payload")
                progress["done"] += 1
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    t0 = time.perf_counter()
    th = [threading.Thread(target=issuer, name="issuer"), threading.Thread(target=completer, name="completer")]
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    print(f"groups {n_groups} issued {progress['issued']} done {progress['done']} in {dt:.2f}s; in_flight {p.in_flight()}; "
          f"errors {errors[:3]}", flush=True)
    p.abort()
    faulthandler.cancel_dump_traceback_later()
    sys.exit(1 if errors or progress["done"] != n_groups or p.in_flight() else 0)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 400)
