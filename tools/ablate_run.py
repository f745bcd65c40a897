"""Time the derivative pass of each ablation variant (same workload, in-kernel stamps)."""
import ctypes, os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1:
    v = sys.argv[1]
    sys.path.insert(0, ROOT)
    import xchu_slam_amd._lib as L
    L.LIB_PATH = os.path.join(ROOT, "build", "ablate", v, "libndt_hip.so")
    import xchu_slam_amd as xa
    from xchu_slam_amd import synth
    c5 = os.environ.get("ABL_WL") == "c5"
    w = synth.make_world(1, half=330.0 if c5 else 210.0)
    pr = synth.make_pair(w, 32.0 if c5 else 8.0, 1_000_000 if c5 else 120000, seed=4, max_range=80.0 if c5 else 60.0)
    g = xa.NormalDistributionsTransform()
    g.setResolution(0.5 if c5 else 1.0)
    g.setTransformationEpsilon(0.0); g.setMaximumIterations(30)
    g.setInputTarget(pr.target); g.setInputSource(pr.source)
    for _ in range(3): g.align(pr.guess, want_output=False)
    g.setProfiling(True)
    for _ in range(10): g.align(pr.guess, want_output=False)
    print(json.dumps({"variant": v, **g.timings()}))
else:
    for v in ["0", "1", "2", "3"]:
        out = subprocess.run([sys.executable, __file__, v], capture_output=True, text=True, timeout=300)
        print(out.stdout.strip() or out.stderr[-500:])
