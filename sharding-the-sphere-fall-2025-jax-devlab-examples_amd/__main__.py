"""Command line:  python -m stsphere <command> ...

    run CONFIG.yaml [--days D | --nsteps K] [--plot]   run the solver
    info CONFIG.yaml                                   validate config, print sharding + halo plan
    schedule                                           print the reference 4-stage halo schedule
    roofline                                           slide-19 roofline / TT model for MI355X
    plot HISTORY.zarr FIELD OUTDIR [--log] [--products frames,band,six] [--every K]
                                                       sphere frames, equatorial band, six-panel
    ensemble CONFIG.yaml [--members M] [--amplitude A] [--days D | --nsteps K]
                                                       perturbed members of one config on one device
    build                                              compile the gfx950 library
"""
import argparse
import json
import os
import sys


def main(argv=None):
    ap = argparse.ArgumentParser(prog="stsphere")
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("config")
    r.add_argument("--days", type=float)
    r.add_argument("--nsteps", type=int)
    r.add_argument("--plot", action="store_true")
    i = sub.add_parser("info")
    i.add_argument("config")
    sub.add_parser("schedule")
    sub.add_parser("roofline")
    p = sub.add_parser("plot")
    p.add_argument("history")
    p.add_argument("field")
    p.add_argument("outdir")
    p.add_argument("--log", action="store_true")
    p.add_argument("--products", default="frames,band,six")
    p.add_argument("--every", type=int, default=1)
    en = sub.add_parser("ensemble")
    en.add_argument("config")
    en.add_argument("--members", type=int, default=2)
    en.add_argument("--amplitude", type=float, default=1e-4)
    en.add_argument("--days", type=float)
    en.add_argument("--nsteps", type=int)
    sub.add_parser("build")
    a = ap.parse_args(argv)

    if a.cmd == "build":
        from .ops import build
        for v in sorted(build.VARIANT_FLAGS):
            print(build.build(force=True, variant=v))
        return 0
    if a.cmd == "schedule":
        from .ops.halo import make_halo_exchange
        from .parallel.topology import create_communication_schedule
        make_halo_exchange(create_communication_schedule(), 4)
        return 0
    if a.cmd == "roofline":
        from .utils.roofline import report
        print(report())
        return 0
    if a.cmd == "plot":
        from .utils.viz import history_products
        for f in history_products(a.history, a.field, a.outdir, log=a.log, every=a.every,
                                  products=tuple(a.products.split(","))):
            print(f)
        return 0
    if a.cmd == "ensemble":
        print(json.dumps(run_ensemble(a.config, a.members, a.amplitude, a.days, a.nsteps), default=float))
        return 0
    from .utils.config import load_config
    if a.cmd == "run" and load_config(a.config).physics.model == "planar_swe":
        from .models.planar import run_panel      # single flat panel, no halos
        print(json.dumps(run_panel(a.config), default=float))
        return 0
    from .driver import Solver
    s = Solver(a.config)
    if a.cmd == "info":
        s.setup_sharding()
        from .parallel.layout import TileLayout
        c = s.cfg
        L = TileLayout(c.grid.N, c.parallelization.tiles_per_edge, c.parallelization.num_devices,
                       ng=c.grid.halo, owner=s.sharding.owner)
        for rk in range(L.num_ranks):
            print(L.plan(rk).summary())
        return 0
    s.initialize()
    summary = s.run(nsteps=a.nsteps, days=a.days)
    g = s.gather_global() if a.plot else None     # collective under SPMD
    s.close()                                     # collective under SPMD (exchange rings)
    if s.rank == 0:
        print(json.dumps(summary, default=float))
        if a.plot:
            from .utils.viz import history_products, sphere_plot
            out = s.cfg.io.output_dir
            os.makedirs(out, exist_ok=True)
            hist = os.path.join(out, "history.zarr")
            log = s.physics.name == "diffusion"
            if os.path.exists(os.path.join(hist, ".zgroup")):
                for f in history_products(hist, s.fields[0], os.path.join(out, "plots"), grid=s.grid, log=log,
                                          products=("band", "six")):
                    print(f)
            print(sphere_plot(g[0], s.grid, os.path.join(out, f"{s.fields[0]}_final.png"), log=log))
    return 0


def run_ensemble(config, members: int, amplitude: float, days=None, nsteps=None) -> dict:
    """``members`` perturbed copies of a run configuration stepped together
    on one device (``stsphere.Ensemble``); returns throughput and spread."""
    import math
    import time
    import torch
    from .ensemble import Ensemble
    from .models.geometry import DAY
    from .utils.config import load_config
    c = load_config(config)
    ens = Ensemble.from_config(c, members, amplitude=amplitude)
    if nsteps is None:
        d = days if days is not None else c.time.days
        nsteps = int(math.ceil(d * DAY / ens.dt - 1e-9)) if d is not None else (c.time.nsteps or 1)
    ens.prepare(nsteps)
    before = ens.spread()
    sync = torch.cuda.synchronize if ens.native else (lambda: None)
    sync()
    t0 = time.perf_counter()
    ens.run(nsteps)
    sync()
    wall = time.perf_counter() - t0
    after = ens.spread()
    ens.close()
    cells = 6 * c.grid.N ** 2
    return {"members": members, "steps": nsteps, "dt": ens.dt, "wall_s": wall,
            "aggregate_cell_updates_per_s": members * cells * nsteps / max(wall, 1e-12),
            "native": ens.native, "field0_mean": after["mean"], "field0_spread_rms_initial": before["spread_rms"],
            "field0_spread_rms_final": after["spread_rms"]}


if __name__ == "__main__":
    sys.exit(main())
