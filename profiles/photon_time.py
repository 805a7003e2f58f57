import importlib, sys, time
sys.path.insert(0, '.')
bre = importlib.import_module("beam-radiance-estimate-pbrt_amd")
sc = importlib.import_module("beam-radiance-estimate-pbrt_amd.scene")
s = sc.cornell_scene()
with bre.BeamGather(0, timing=True) as g:
    for it in range(3):
        t = time.time(); nb = g.trace_photons(s, 1_000_000, iteration=it, max_depth=5); dt = time.time() - t
        st = g.stats()
        print(f"iter {it}: beams {nb} wall {dt*1e3:.1f} ms photon_ms {st['photon_ms']:.2f} build_ms {st['build_ms']:.2f}", flush=True)
