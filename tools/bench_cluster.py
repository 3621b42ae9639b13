#!/usr/bin/env python3
"""configs[4]: server.py + GPU-backed client.py processes (one or more per GPU) on one node, Office test
document, -pr 8, payload size per GPU.  Starts `python -m dprf_amd.server` with a bounded keyspace
(--max-candidates, from the start of the -pr 8 order) and the clients, waits for the server to drain, and
prints one JSON line: end-to-end rate (candidates acknowledged / time from the first payload sent to the
last acknowledgement) next to the clients' own GPU-side rates.

Usage (on the GPU box): python tools/bench_cluster.py [--gpus N] [--clients-per-gpu M] [--payload P]
                                                     [--candidates C] [--workload office]
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
DOCS = {"office": "office_testdoc", "odt": "odt_testdoc_std", "pdf_r34": "pdf_testdoc_r4"}


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run(gpus=1, clients_per_gpu=2, payload=1 << 20, candidates=24 << 20, workload="office", builders=4,
        timeout=300, dry_run=False, devices=None):
    """Start the server and the clients, wait for the server to drain; returns the result dict."""
    stream = json.load(open(os.path.join(REPO, "tests", "golden", "streams.json")))[DOCS[workload]]["stream"]
    port, hb = free_port(), free_port()
    env = dict(os.environ)
    env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
    srv = subprocess.Popen([sys.executable, "-m", "dprf_amd.server", "1", "unused.docx", "-pr", "8", "-ps",
                            str(payload), "127.0.0.1", str(port), "--stream", stream, "--max-candidates",
                            str(candidates), "--heartbeat-port", str(hb), "--quiet", "--builders",
                            str(builders)], cwd=REPO, env=env, stdout=subprocess.PIPE, text=True)
    for _ in range(100):                       # wait for the work port
        try:
            socket.create_connection(("127.0.0.1", port), timeout=0.2).close()
            break
        except OSError:
            time.sleep(0.1)
    # (the server ignores the empty probe connection)
    clients = []
    for g in (devices if devices is not None else range(gpus)):
        for _ in range(clients_per_gpu):
            cenv = dict(env)
            cenv["HIP_VISIBLE_DEVICES"] = str(g)
            clients.append(subprocess.Popen([sys.executable, "-m", "dprf_amd.client", "127.0.0.1", str(port),
                                             "--devices", "0", "--quiet", "--heartbeat-port", str(hb)]
                                            + (["--dry-run"] if dry_run else []),
                                            cwd=REPO, env=cenv, stdout=subprocess.PIPE, text=True))
    t0 = time.time()
    try:
        out, _ = srv.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        srv.kill()
        for c in clients:
            c.kill()
        raise
    res = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    couts = []
    for c in clients:
        o, _ = c.communicate(timeout=60)
        couts += [json.loads(l) for l in o.splitlines() if l.startswith("{")]
    s = res[-1] if res else {}
    return {"metric": "end-to-end verified candidates/sec, server.py + GPU client.py (configs[4])"
                      + (" -- DRY RUN: clients verify nothing" if dry_run else ""),
            "workload": workload, "n_gpus": gpus, "clients": len(clients), "payload": payload,
            "candidates": s.get("acknowledged"), "value": s.get("rate"), "unit": "candidates/s",
            "server_from_first_payload_s": s.get("from_first_payload_s"),
            "client_verified": sum(c["verified"] for c in couts),
            "clients_detail": couts, "wall_s": time.time() - t0, "complete": s.get("acknowledged") == candidates}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--clients-per-gpu", type=int, default=2)
    ap.add_argument("--payload", type=int, default=1 << 20)
    ap.add_argument("--candidates", type=int, default=24 << 20)
    ap.add_argument("--workload", default="office", choices=sorted(DOCS))
    ap.add_argument("--builders", type=int, default=4)
    ap.add_argument("--timeout", type=float, default=300)
    ap.add_argument("--dry-run", action="store_true", help="clients parse payloads but verify nothing (no GPU)")
    args = ap.parse_args()
    line = run(args.gpus, args.clients_per_gpu, args.payload, args.candidates, args.workload, args.builders,
               args.timeout, args.dry_run)
    print(json.dumps(line), flush=True)
    return 0 if line["complete"] else 1


if __name__ == "__main__":
    sys.exit(main())
