"""Worker for tests/test_gpu_xgmi.py: a real multi-rank RCCL data plane on ONE GPU.

    RANK=r WORLD_SIZE=2 MASTER_PORT=p NCCL_HOSTID=p2pfl-r<r> python tests/rccl_worker.py OUT_JSON

RCCL refuses two ranks of one communicator on the same device ("Duplicate GPU
detected") unless they look like different hosts: a distinct ``NCCL_HOSTID``
per rank makes each rank its own "host", so the communicator forms over RCCL's
network transport (sockets on loopback) instead of xGMI peer-to-peer.  The
bytes then travel GPU -> host -> socket -> host -> GPU, so this measures
nothing about xGMI; what it exercises for real is everything above the wire:
multi-rank non-blocking communicator init from a store-exchanged unique id,
the epoch-grouped schedule with both ranks pushing to each other at the same
moment (send and receive of one epoch in ONE ncclGroupStart/End on each rank),
producer-event ordering on the comm stream, completion polling, and the
native binding's locking under the data plane's issuer/completer threads.
"""

from __future__ import annotations

import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def _say(msg: str) -> None:
    print(f"[rccl_worker {os.environ.get('RANK')}] {time.strftime('%H:%M:%S')} {msg}", flush=True)


def main(out: str) -> None:
    import faulthandler

    faulthandler.dump_traceback_later(float(os.environ.get("P2PFL_WORKER_WATCHDOG", "100")), exit=True)
    from p2pfl_amd.communication.xgmi.data_plane import XgmiDataPlane, make_backend_factory

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    store = dist.TCPStore("127.0.0.1", int(os.environ["MASTER_PORT"]), world, rank == 0, wait_for_workers=False)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    plane = XgmiDataPlane(rank, world, make_backend_factory("rccl", rank, store, "r2", dev, timeout=60.0),
                          store=store, prefix="r2", device=dev, ack_timeout=30.0, group_timeout=60.0, preconnect=True)
    plane.allow_fallback = False
    t0 = time.perf_counter()
    _say("communicator init")
    plane.start(block=True)
    init_s = time.perf_counter() - t0
    _say(f"plane up in {init_s:.2f}s: backend {plane.backend_name}, failed={plane.failed}")
    if plane.failed:
        raise SystemExit(f"rank {rank}: {plane.failed}")
    peer = 1 - rank
    n, pushes = 6_497_280, 6  # CNN-sized fp32 arenas
    lock = threading.Lock()
    received, sent_ok = [], []
    done = threading.Semaphore(0)

    # header exchange through the store (the transport uses the control bus).
    # A TCPStore client holds its connection lock for the whole of a blocking
    # get(), so every thread that waits on a key gets its own client.
    def client():
        return dist.TCPStore("127.0.0.1", int(os.environ["MASTER_PORT"]), world, False)

    def serve_headers():
        st = client()
        for i in range(pushes):
            hdr = json.loads(st.get(f"hdr/{peer}/{i}").decode())

            def on_recv(buf, reason, i=i):
                with lock:
                    received.append((i, None if buf is None else buf.clone(), reason))
                done.release()

            e, why = plane.accept(peer, hdr, on_recv)
            assert e is not None, why
            st.set(f"ack/{peer}/{i}", json.dumps([hdr["seq"], e, hdr["gen"]]))

    def collect_acks(seqs):
        st = client()
        for i in range(pushes):
            seq, e, gen = json.loads(st.get(f"ack/{rank}/{i}").decode())
            plane.on_ack(seq, e, gen)

    srcs = []
    server = threading.Thread(target=serve_headers, daemon=True)
    server.start()
    seqs = []
    for i in range(pushes):
        t = torch.empty(n, device=dev)
        t.copy_(torch.arange(n, device=dev, dtype=torch.float32) * 1e-3 + (rank * 100 + i))  # produced by a kernel
        srcs.append(t)

        def on_send(ok, reason, evict, i=i):
            with lock:
                sent_ok.append((i, ok, reason))
            done.release()

        hdr = plane.propose(peer, t, on_send)
        seqs.append(hdr["seq"])
        store.set(f"hdr/{rank}/{i}", json.dumps(hdr))
    acker = threading.Thread(target=collect_acks, args=(seqs,), daemon=True)
    acker.start()
    _say(f"{pushes} pushes proposed")
    t1 = time.perf_counter()
    for k in range(2 * pushes):
        if not done.acquire(timeout=60):
            _say(f"stalled after {k} completions; stats {dict(plane.stats)}")
            raise SystemExit(f"rank {rank}: transfers stalled")
    xfer_s = time.perf_counter() - t1
    _say(f"transfers done in {xfer_s:.3f}s; stats {dict(plane.stats)}")
    ok = all(o for _, o, _ in sent_ok) and len(sent_ok) == pushes
    bad = []
    for i, buf, reason in received:
        exp = torch.arange(n, device=dev, dtype=torch.float32) * 1e-3 + (peer * 100 + i)
        if buf is None or not torch.equal(buf, exp):
            bad.append((i, reason))
    stats = dict(plane.stats)
    store.set(f"fin/{rank}", "1")
    store.wait([f"fin/{r}" for r in range(world)])
    plane.stop()
    with open(f"{out}.{rank}", "w") as f:
        json.dump({"rank": rank, "sends_ok": ok, "received": len(received), "bad": bad, "stats": stats,
                   "init_s": init_s, "xfer_s": xfer_s, "backend": plane.backend_name}, f)


if __name__ == "__main__":
    main(sys.argv[1])
