"""Pipelined contexts on one device (include/bre.h: bre_set_gather_after, bre_set_gather_events,
bre_film_add; bench.py's two-context step).  Two contexts on two streams, each linked after the other,
render alternate iterations into their own films and add them into one film: the film must be the same
bits as the same iterations rendered one after another on one unlinked context.  Destroying a context
unlinks its partner (its later gathers no longer wait on a freed event), and the timing events bracket
the tile kernels only (elapsed > 0 and below the whole gather's)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W = H = 64
PHOTONS = 20_000


def _iteration(bre, g, scene, it, film, surf):
    R = bre.beam_radius_at(0.01, 0.5, it)
    g.trace_photons(scene, PHOTONS, it, 5, R)
    g.camera_pass(scene, W, H, it, 5, True, True, surface=surf)
    g.gather_camera(R, film)


def _serial(bre, scene, iters):
    import torch

    film = torch.zeros((W * H, 3), dtype=torch.float32, device="cuda")
    surf = torch.zeros_like(film)
    with bre.BeamGather(0) as g:
        st = torch.cuda.Stream()
        g.set_stream(st.cuda_stream)
        with torch.cuda.stream(st):
            for it in iters:
                part = torch.zeros_like(film)
                _iteration(bre, g, scene, it, part, surf)
                g.film_add(part, film, clear_src=True)
        st.synchronize()
    return film.cpu().numpy(), surf.cpu().numpy()


def test_linked_contexts_give_the_serial_film(bre, scene_mod_gpu):
    import torch

    scene = scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0)
    iters = [1, 2, 3, 4]
    ref_film, ref_surf = _serial(bre, scene, iters)

    film = torch.zeros((W * H, 3), dtype=torch.float32, device="cuda")
    surf = [torch.zeros_like(film), torch.zeros_like(film)]
    parts = [torch.zeros_like(film), torch.zeros_like(film)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    a, b = bre.BeamGather(0), bre.BeamGather(0)
    try:
        for g, st in zip((a, b), streams):
            g.set_stream(st.cuda_stream)
        a.set_gather_after(b)
        b.set_gather_after(a)
        done = [None, None]
        for k, it in enumerate(iters):
            i = k % 2
            g, st = (a, b)[i], streams[i]
            with torch.cuda.stream(st):
                if k >= 1:  # film adds happen in iteration order: wait for the previous one
                    st.wait_event(done[1 - i])
                _iteration(bre, g, scene, it, parts[i], surf[i])
                g.film_add(parts[i], film, clear_src=True)
                done[i] = torch.cuda.Event()
                done[i].record(st)
        torch.cuda.synchronize()
    finally:
        b.set_gather_after(None)
        a.close()
        b.close()
    assert np.array_equal(film.cpu().numpy(), ref_film)
    # the surface (direct) term: iterations split over two accumulators, summed in the same order per
    # pixel only when each pixel sees one nonzero add -- compare the sum with a tolerance instead
    s = (surf[0] + surf[1]).cpu().numpy()
    assert np.allclose(s, ref_surf, rtol=1e-5, atol=1e-6)


def test_destroying_the_leader_unlinks(bre, scene_mod_gpu):
    import torch

    scene = scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0)
    ref_film, _ = _serial(bre, scene, [3])
    a, b = bre.BeamGather(0), bre.BeamGather(0)
    try:
        film = torch.zeros((W * H, 3), dtype=torch.float32, device="cuda")
        surf = torch.zeros_like(film)
        _iteration(bre, a, scene, 1, torch.zeros_like(film), torch.zeros_like(film))
        a.synchronize()
        b.set_gather_after(a)
        a.close()  # bre_destroy(a) clears b's link to a's event
        _iteration(bre, b, scene, 3, film, surf)
        b.synchronize()
        assert np.array_equal(film.cpu().numpy(), ref_film)
    finally:
        a.close()
        b.close()


def test_gather_after_self_is_refused(bre):
    with bre.BeamGather(0) as g:
        with pytest.raises(Exception):
            g.set_gather_after(g)


def test_gather_events_bracket_the_tile_kernel(bre, scene_mod_gpu):
    import torch

    scene = scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0)
    st = torch.cuda.Stream()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    w0, w1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for e in (t0, t1, w0, w1):
        e.record(st)  # so that the HIP events exist
    st.synchronize()
    with bre.BeamGather(0) as g:
        g.set_stream(st.cuda_stream)
        g.set_gather_events(t0, t1)
        R = bre.beam_radius_at(0.01, 0.5, 1)
        film = torch.zeros((W * H, 3), dtype=torch.float32, device="cuda")
        with torch.cuda.stream(st):
            g.trace_photons(scene, PHOTONS, 1, 5, R)
            g.camera_pass(scene, W, H, 1, 5, True, True, surface=torch.zeros_like(film))
            w0.record(st)
            g.gather_camera(R, film)
            w1.record(st)
        st.synchronize()
        g.set_gather_events(None, None)
    tile, whole = t0.elapsed_time(t1), w0.elapsed_time(w1)
    assert 0.0 < tile <= whole


def test_coarse_sort_keys_keep_every_pair(bre, scene_mod_gpu):
    """Internal option 121 (1; default 0): the tree-order and segment sorts use the keys' top 48 bits.  Only
    orders change (the tree's leaf tiles, the packets), so every segment keeps its contribution count and
    its sum to float summation order, in camera-pass order."""
    import torch

    scene = scene_mod_gpu.cornell_scene(0.05, 0.5, 0.0)
    R = bre.beam_radius_at(0.01, 0.5, 2)
    outs = {}
    for coarse in (0, 1):
        with bre.BeamGather(0) as g:
            g.set_option(121, coarse)
            g.trace_photons(scene, 100_000, 2, 5, R)
            n = g.camera_pass(scene, 128, 128, 2, 5, True, True)
            rgb = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
            cnt = torch.zeros((n, 2), dtype=torch.int32, device="cuda")
            g.gather_camera_segments(R, seg_rgb=rgb, counts=cnt)
            g.synchronize()
            outs[coarse] = (rgb.cpu().numpy(), cnt.cpu().numpy())
    assert outs[0][1][:, 1].sum() > 0
    assert np.array_equal(outs[0][1][:, 1], outs[1][1][:, 1])
    c = outs[0][1][:, 1].astype(np.float64)
    tol = np.maximum(1e-5, 4 * 2.0 ** -24 * np.sqrt(np.maximum(c, 1)))[:, None]
    assert (np.abs(outs[1][0] - outs[0][0]) <= tol * np.maximum(np.abs(outs[0][0]), 1e-30)).all()
