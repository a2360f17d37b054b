#!/usr/bin/env python
"""Solver.run overhead probe (GPU): the C48 config with the I/O intervals
switched on one at a time, so each phase's cost on the stepping throughput
shows against pure stepping.

    python tools/run_phase_probe.py [--days 2] [--out DIR]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--days", type=float, default=2.0)
    ap.add_argument("--out", default="gpurun_out/phase_probe")
    a = ap.parse_args()
    import yaml
    from stsphere.driver import Solver
    base = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "sharding-the-sphere-fall-2025-jax-devlab-examples_amd", "configs", "c48_1gpu.yaml")
    cfg0 = yaml.safe_load(open(base))
    variants = {
        "stepping_only": dict(history_interval=0, checkpoint_interval=0, metrics_interval=0, watchdog=0),
        "watchdog_96": dict(history_interval=0, checkpoint_interval=0, metrics_interval=0, watchdog=96),
        "metrics_96": dict(history_interval=0, checkpoint_interval=0, metrics_interval=96, watchdog=0),
        "history_288": dict(history_interval=288, checkpoint_interval=0, metrics_interval=0, watchdog=0),
        "config_as_shipped": dict(history_interval=288, checkpoint_interval=1440, metrics_interval=96, watchdog=96),
    }
    res = {}
    for name, v in variants.items():
        cfg = json.loads(json.dumps(cfg0))
        out = os.path.join(a.out, name)
        cfg["io"].update(output_dir=out, history_interval=v["history_interval"],
                         checkpoint_interval=v["checkpoint_interval"], metrics_interval=v["metrics_interval"])
        cfg["io"].pop("geometry", None)
        cfg["io"].pop("initial_condition", None)
        cfg["runtime"] = dict(cfg.get("runtime", {}), watchdog_interval=v["watchdog"])
        s = Solver(cfg, verbose=False)
        s.initialize()
        r = s.run(days=a.days)
        res[name] = {"us_per_step": 1e6 * r["wall_s"] / r["steps_run"], "cell_updates_per_s": r["cell_updates_per_s"],
                     "phase_s": r["phase_s"], "steps": r["steps_run"]}
        print(name, json.dumps(res[name]), flush=True)
    os.makedirs(a.out, exist_ok=True)
    json.dump(res, open(os.path.join(a.out, "phase_probe.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
