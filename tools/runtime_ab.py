"""A/B of the step runtimes on one engine config, interleaved in one process:
native C++ runtime (hipGraph) on a normal / high-priority stream,
and torch.cuda.graph replay (GraphStepper)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from stsphere.engine import Engine, GraphStepper
from stsphere.models.geometry import CubedSphereGrid
from stsphere.models.swe import ShallowWater
from stsphere.ops.native_runtime import NativeStepper
from stsphere.parallel.layout import TileLayout

N = int(os.environ.get("N", "96"))
g = CubedSphereGrid(N)
L = TileLayout(N, 2, 1, ng=2)


def mk():
    return Engine(ShallowWater("tc5"), L, grid=g, device="cuda", backend="hip")


class TorchCapturedNative:
    """The native runtime's eager op list, recorded by torch.cuda.graph."""

    def __init__(self, e, k=30):
        self.s = torch.cuda.Stream()
        self.ns = NativeStepper(e, use_graph=False, stream=self.s)
        self.ns.run(1)
        torch.cuda.synchronize()
        self.k = k
        self.g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g, stream=self.s):
            self.ns.L.stsp_rt_run(self.ns.h, k)

    def run(self, n):
        for _ in range(n // self.k):
            self.g.replay()


runners = {
    "native_eager": NativeStepper(mk(), use_graph=False),
    "native_in_torch_graph": TorchCapturedNative(mk()),
    "native_default": NativeStepper(mk(), use_graph=True, steps_per_graph=30),
    "native_cxx_graph": None,
    "torch_graph": GraphStepper(mk(), 30),
}
os.environ["STSP_NATIVE_GRAPH"] = "1"
runners["native_cxx_graph"] = NativeStepper(mk(), use_graph=True, steps_per_graph=30)
os.environ.pop("STSP_NATIVE_GRAPH")
for r in runners.values():
    r.run(60)
torch.cuda.synchronize()
res = {k: [] for k in runners}
host = {k: [] for k in runners}
for rnd in range(3):
    for k, r in runners.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.run(600)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        res[k].append((time.perf_counter() - t0) / 600 * 1e6)
        host[k].append((t1 - t0) / 600 * 1e6)
print(json.dumps({"us_per_step": {k: [round(x, 2) for x in v] for k, v in res.items()},
                  "host_us_per_step_until_return": {k: [round(x, 2) for x in v] for k, v in host.items()}}))
