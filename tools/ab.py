"""Interleaved A/B of bench.py under environment variants, on one GPU box.

    python tools/ab.py --rounds 3 --bench=--workload,c5,--no-cpu,--alt-steps,0 \
        --variant base= --variant roll=GMAGG_PASS_VARIANT=2 [--out gpurun_out/x/ab.jsonl]

Each round runs every variant once (a fresh bench.py process each, in variant order), so
box drift hits every variant alike (cdna_hip_programming.md §5.4 rule 24).  Prints one
JSON line per run and a per-variant summary (median / min / max of the bench value and of
the dominant kernel's average launch time).  A variant is NAME=[VAR=VALUE[;VAR=VALUE...]];
--bench is bench.py's arguments separated by commas (no shell quoting needed).
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--bench", default="")
    ap.add_argument("--variant", action="append", default=[])
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    variants = []
    for v in a.variant or ["base="]:
        name, _, envs = v.partition("=")
        env = {}
        for kv in filter(None, envs.split(";")):
            k, _, val = kv.partition("=")
            env[k] = val
        variants.append((name, env))
    runs = {name: [] for name, _ in variants}
    out = open(a.out, "a") if a.out else None
    for r in range(a.rounds):
        for name, env in variants:
            e = dict(os.environ, **env)
            cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + [x for x in a.bench.split(",") if x]
            p = subprocess.run(cmd, env=e, capture_output=True, text=True, timeout=a.timeout)
            if p.returncode != 0:
                sys.stderr.write(p.stderr[-3000:])
                raise SystemExit(f"variant {name} round {r}: bench.py exited {p.returncode}")
            line = json.loads(p.stdout.strip().splitlines()[-1])
            roof = line.get("roofline") or {}
            rec = {"variant": name, "round": r, "value": line["value"],
                   "ms_per_step": line["ms_per_step"], "avg_launch_us": roof.get("avg_launch_us"),
                   "frac": roof.get("frac"), "aggregation_frac": roof.get("aggregation_frac"),
                   "groups": (line.get("config") or {}).get("groups")}
            runs[name].append(rec)
            s = json.dumps(rec)
            print(s, flush=True)
            if out:
                out.write(s + "\n")
                out.flush()
    for name, recs in runs.items():
        vals = [x["value"] for x in recs]
        us = [x["avg_launch_us"] for x in recs if x["avg_launch_us"]]
        summ = {"variant": name, "value_median": statistics.median(vals), "value_min": min(vals),
                "value_max": max(vals),
                "launch_us_median": statistics.median(us) if us else None}
        print(json.dumps(summ), flush=True)
        if out:
            out.write(json.dumps(summ) + "\n")


if __name__ == "__main__":
    main()
