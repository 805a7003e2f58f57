"""MI355X beam-radiance-estimate gather — Python bindings over the C ABI of libbre.so.

The product is the C ABI in ``include/bre.h`` (libbre.so, hand-written HIP for gfx950).  This
module is a thin ctypes binding used by the tests, ``bench.py`` and ``__graft_entry__``; it has
no compute of its own and no CPU fallback: if libbre.so is missing or no GPU is present, the
calls fail loudly.

Import with ``importlib.import_module("beam-radiance-estimate-pbrt_amd")`` (the directory name
is not a Python identifier) or via ``tests/conftest.py``'s ``bre`` fixture.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# BRE_LIBRARY: another build of the same C ABI (profiling ablations, profiles/ablate.sh); the
# default is the in-tree libbre.so.  There is no CPU fallback either way.
LIB_PATH = os.environ.get("BRE_LIBRARY") or os.path.join(HERE, "libbre.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "bre.h")

BRE_OK = 0
STATUS_NAMES = {0: "BRE_OK", 1: "BRE_ERR_INVALID_ARG", 2: "BRE_ERR_HIP", 3: "BRE_ERR_OOM",
                4: "BRE_ERR_STATE", 5: "BRE_ERR_NO_DEVICE"}
OPT_COUNTERS, OPT_TIMING, OPT_KERNEL, OPT_LEAF_SIZE, OPT_SQRT_MODE, OPT_SPLIT, OPT_PREFILTER = 1, 2, 3, 4, 5, 6, 7
OPT_SHARD_RANK, OPT_SHARD_COUNT, OPT_TILE_LEAF = 8, 9, 10
OPT_CHUNK_LEN, OPT_CHUNK_LEAF, OPT_SORT_SEGMENTS, OPT_SHARD_BLOCK, OPT_SHARD_MODE = 11, 12, 13, 14, 15
OPT_FILM_CLASSES, FILM_CLASSES = 16, 8
EMPTY_CHILD = -(2 ** 31)  # kEmptyChild (bre_device.h): no child

# Every entry point include/bre.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "bre_abi_version", "bre_create", "bre_destroy", "bre_last_error", "bre_set_option",
    "bre_set_stream", "bre_synchronize", "bre_get_stats", "bre_set_beams",
    "bre_set_beams_device", "bre_gather", "bre_gather_device", "bre_beam_radius_at",
    "bre_resolve_image", "bre_trace_photons", "bre_get_beams", "bre_scene_cornell", "bre_scene_cornell_smoke", "bre_smoke_density",
    "bre_camera_pass", "bre_gather_camera", "bre_gather_camera_segments", "bre_get_segments",
    "bre_render_iteration", "bre_render",
    "bre_render_progressive", "bre_shard_segments", "bre_set_beams_sharded", "bre_gather_sharded",
    "bre_device_check", "bre_resolve_classes", "bre_film_add", "bre_set_gather_after", "bre_set_gather_events",
]


class BreError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class Stats(ctypes.Structure):
    _fields_ = [("n_beams", ctypes.c_int64), ("n_beams_valid", ctypes.c_int64),
                ("n_nodes", ctypes.c_int64), ("n_segments", ctypes.c_int64),
                ("candidates", ctypes.c_int64), ("contributions", ctypes.c_int64),
                ("node_visits", ctypes.c_int64), ("leaf_visits", ctypes.c_int64),
                ("beam_evals", ctypes.c_int64), ("ccp_wave_evals", ctypes.c_int64),
                ("prefilter_rejects", ctypes.c_int64), ("useful_beam_evals", ctypes.c_int64),
                ("max_stack_depth", ctypes.c_int64), ("redo_items", ctypes.c_int64),
                ("build_ms", ctypes.c_double),
                ("gather_ms", ctypes.c_double),
                ("n_photons", ctypes.c_int64),
                ("photon_ms", ctypes.c_double),
                ("n_camera_segments", ctypes.c_int64),
                ("camera_ms", ctypes.c_double), ("n_chunks", ctypes.c_int64),
                ("queued_pairs", ctypes.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_LIB = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libbre.so and declare its signatures.  Raises if it is not built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    # PyTorch-ROCm bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's).  Whichever is
    # loaded first serves the whole process, and torch cannot initialise on a runtime it was not
    # built with, so load torch's first whenever torch is installed (it is the process's
    # allocator / stream / RCCL plumbing in bench.py and the device-pointer tests).
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not found: build it with `make -C {HERE}/csrc` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(path)
    P, I64, I32, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float
    lib.bre_abi_version.restype = I32
    lib.bre_create.argtypes = [I32, ctypes.POINTER(P)]
    lib.bre_create.restype = I32
    lib.bre_destroy.argtypes = [P]
    lib.bre_destroy.restype = None
    lib.bre_last_error.argtypes = [P]
    lib.bre_last_error.restype = ctypes.c_char_p
    lib.bre_set_option.argtypes = [P, I32, I64]
    lib.bre_set_option.restype = I32
    lib.bre_set_stream.argtypes = [P, P]
    lib.bre_set_stream.restype = I32
    lib.bre_synchronize.argtypes = [P]
    lib.bre_synchronize.restype = I32
    lib.bre_get_stats.argtypes = [P, ctypes.POINTER(Stats)]
    lib.bre_get_stats.restype = I32
    for fn in (lib.bre_set_beams, lib.bre_set_beams_device):
        fn.argtypes = [P, I64, P, P, P, P]
        fn.restype = I32
    for fn in (lib.bre_gather, lib.bre_gather_device):
        fn.argtypes = [P, I64, P, P, P, P, P, F, I64, P, P, P]
        fn.restype = I32
    lib.bre_beam_radius_at.argtypes = [F, F, I32]
    lib.bre_beam_radius_at.restype = F
    lib.bre_shard_segments.argtypes = [I64, I32, I32, I32]
    lib.bre_shard_segments.restype = I64
    lib.bre_resolve_image.argtypes = [I64, P, I32, P]
    lib.bre_resolve_image.restype = I32
    lib.bre_trace_photons.argtypes = [P, P, I64, I32, I32, F, ctypes.POINTER(I64)]
    lib.bre_trace_photons.restype = I32
    lib.bre_get_beams.argtypes = [P, I64, P, P, P, P, ctypes.POINTER(I64)]
    lib.bre_get_beams.restype = I32
    lib.bre_scene_cornell.argtypes = [P, F, F, F]
    lib.bre_scene_cornell.restype = None
    lib.bre_scene_cornell_smoke.argtypes = [P, F, F, F, I32, P]
    lib.bre_scene_cornell_smoke.restype = None
    lib.bre_smoke_density.argtypes = [I32, ctypes.c_uint64, P]
    lib.bre_smoke_density.restype = None
    lib.bre_camera_pass.argtypes = [P, P, I32, I32, I32, I32, I32, I32, P, ctypes.POINTER(I64)]
    lib.bre_camera_pass.restype = I32
    lib.bre_gather_camera.argtypes = [P, F, P]
    lib.bre_gather_camera.restype = I32
    lib.bre_gather_camera_segments.argtypes = [P, F, P, P, P]
    lib.bre_gather_camera_segments.restype = I32
    lib.bre_get_segments.argtypes = [P, I64, P, P, P, P, P, P, ctypes.POINTER(I64)]
    lib.bre_get_segments.restype = I32
    lib.bre_render_iteration.argtypes = [P, P, P, I32, P]
    lib.bre_render_iteration.restype = I32
    lib.bre_render.argtypes = [P, P, P, P]
    lib.bre_render.restype = I32
    lib.bre_render_progressive.argtypes = [P, P, P, I32, P, P]
    lib.bre_render_progressive.restype = I32
    lib.bre_set_beams_sharded.argtypes = [P, I32, I64, P, P, P, P]
    lib.bre_set_beams_sharded.restype = I32
    lib.bre_gather_sharded.argtypes = [P, I32, I64, P, P, P, P, P, F, I64, P, P, P]
    lib.bre_gather_sharded.restype = I32
    if hasattr(lib, "bre_resolve_classes"):  # (absent from round-4 libraries loaded for A/B timing)
        lib.bre_resolve_classes.argtypes = [P, I64, P, P]
        lib.bre_resolve_classes.restype = I32
    if hasattr(lib, "bre_film_add"):  # (absent from round-5 libraries loaded for A/B timing)
        lib.bre_film_add.argtypes = [P, I64, P, P, I32]
        lib.bre_film_add.restype = I32
        lib.bre_set_gather_after.argtypes = [P, P]
        lib.bre_set_gather_after.restype = I32
        lib.bre_set_gather_events.argtypes = [P, P, P]
        lib.bre_set_gather_events.restype = I32
    if hasattr(lib, "bre_device_check"):  # (absent from round-3 libraries loaded for A/B timing)
        lib.bre_device_check.argtypes = [P, I32, I64, P, I32, P, P]
        lib.bre_device_check.restype = I32
    _LIB = lib
    return lib


def _ptr(a):
    """Raw pointer of a numpy array or a torch tensor (None -> NULL)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()  # torch tensor


def _check_device_f32(t, what: str):
    """A device buffer handed to libbre as a raw pointer must be a contiguous float32 CUDA tensor: the
    library reads and writes it as float[] on the device, so anything else is refused before a launch."""
    import torch

    if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
        desc = (f"{t.dtype} on {t.device}, contiguous={t.is_contiguous()}" if isinstance(t, torch.Tensor)
                else type(t).__name__)
        raise ValueError(f"{what}: needs a contiguous float32 CUDA tensor, got {desc}")


def _f32(a, n3=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a


class BeamGather:
    """One libbre context on one GPU (mirrors the life of one PhotonBeamBVH + gather loop)."""

    def __init__(self, device: int = 0, counters: bool = False, timing: bool = False, kernel: int = 0,
                 leaf_size: int | None = None, sqrt_mode: int = 0, split: int | None = None,
                 prefilter: bool | None = None):
        self.lib = load_library()
        h = ctypes.c_void_p()
        st = self.lib.bre_create(device, ctypes.byref(h))
        if st != BRE_OK:
            raise BreError(st, f"bre_create(device={device}) failed")
        self.h = h
        self.set_option(OPT_COUNTERS, int(counters))
        self.set_option(OPT_TIMING, int(timing))
        self.set_option(OPT_KERNEL, kernel)
        self.set_option(OPT_SQRT_MODE, sqrt_mode)
        if leaf_size is not None:
            self.set_option(OPT_LEAF_SIZE, leaf_size)
        if split is not None:
            self.set_option(OPT_SPLIT, split)
        if prefilter is not None:
            self.set_option(OPT_PREFILTER, int(prefilter))
        self._keep = []

    _classes = 1  # BRE_OPT_FILM_CLASSES as set through this wrapper
    _cam_npix = 0  # pixels of the last camera pass

    def _check(self, st):
        if st != BRE_OK:
            raise BreError(st, self.lib.bre_last_error(self.h).decode())

    def set_option(self, opt: int, value: int):
        self._check(self.lib.bre_set_option(self.h, opt, int(value)))
        if opt == OPT_FILM_CLASSES:
            self._classes = int(value)

    def set_shard(self, rank: int, count: int, block: int = 1, packets: bool = False, roots: bool = False):
        """Tile shards (default): the camera pass walks only the 16x16 image tiles of the blocks of
        block x block tiles whose row-major block index is rank (mod count) (dist.tile_pixels lists the
        same pixels).  packets=True: the whole camera pass, and the gather of this rank's chunks of
        `block` consecutive sorted packets, chunk c to rank c mod count (shard_packet_index); the ranks'
        films sum to the whole film.  roots=True (BRE_OPT_SHARD_MODE 2): the whole camera pass, and the
        gather of every segment against this rank's work roots (rank, rank + count, ... of the
        size-ordered list); the ranks' films sum to the whole film."""
        self.set_option(OPT_SHARD_MODE, 2 if roots else (1 if packets else 0))
        self.set_option(OPT_SHARD_BLOCK, int(block))
        self.set_option(OPT_SHARD_COUNT, int(count))
        self.set_option(OPT_SHARD_RANK, int(rank))

    def set_film_classes(self, classes: int):
        """BRE_OPT_FILM_CLASSES: 1 (one film) or FILM_CLASSES (8 planes per film, see include/bre.h)."""
        self.set_option(OPT_FILM_CLASSES, int(classes))

    def _film(self, buf, npix: int, what: str):
        """A caller film must hold classes * 3 * npix floats: the library writes plane p % classes of
        pixel p through a raw pointer, so a short buffer is refused here, before any launch."""
        if buf is None:
            return None
        need = self._classes * 3 * int(npix)
        n = buf.numel() if hasattr(buf, "numel") else int(np.asarray(buf).size)
        if n < need:
            raise ValueError(f"{what}: film of {n} floats, the context's {self._classes} film class(es) over "
                             f"{npix} pixels need {need}")
        _check_device_f32(buf, what)
        return buf

    def resolve_classes(self, classes, out):
        """out (npix, 3) = the sum of the 8 class planes of `classes` ((8 * npix, 3) or (8, npix, 3),
        torch CUDA float32), added in class order on the context's stream."""
        _check_device_f32(classes, "resolve_classes: classes")
        _check_device_f32(out, "resolve_classes: out")
        npix = out.numel() // 3
        if classes.numel() != FILM_CLASSES * 3 * npix:
            raise ValueError(f"resolve_classes: {classes.numel()} floats of class planes for {npix} pixels, "
                             f"need {FILM_CLASSES * 3 * npix}")
        self._check(self.lib.bre_resolve_classes(self.h, npix, _ptr(classes), _ptr(out)))

    def film_add(self, src, dst, clear_src: bool = False):
        """dst += src (torch CUDA float32 tensors of one size), then src = 0 if clear_src, on the
        context's stream (bre_film_add: a one-wave kernel that runs beside another context's gather)."""
        _check_device_f32(src, "film_add src")
        _check_device_f32(dst, "film_add dst")
        if src.numel() != dst.numel():
            raise ValueError(f"film_add: {src.numel()} vs {dst.numel()} floats")
        self._check(self.lib.bre_film_add(self.h, src.numel(), _ptr(src), _ptr(dst), int(bool(clear_src))))

    def set_gather_after(self, prev: "BeamGather | None"):
        """bre_set_gather_after: this context's tile kernels start after prev's last one (pipelined
        contexts on one device; None clears)."""
        self._after = prev  # bre_destroy(prev) unlinks; the reference keeps prev from being collected first
        self._check(self.lib.bre_set_gather_after(self.h, prev.h if prev is not None else None))

    def set_gather_events(self, start=None, end=None):
        """bre_set_gather_events: torch.cuda.Event pair (enable_timing, already recorded once so that the
        HIP event exists) recorded by libbre around the tile kernel of every later gather; None clears."""
        h = lambda e: None if e is None else int(e.cuda_event)  # noqa: E731
        self._check(self.lib.bre_set_gather_events(self.h, h(start), h(end)))

    def set_stream(self, stream_handle: int | None):
        self._check(self.lib.bre_set_stream(self.h, stream_handle))

    def synchronize(self):
        self._check(self.lib.bre_synchronize(self.h))

    def stats(self) -> dict:
        s = Stats()
        self._check(self.lib.bre_get_stats(self.h, ctypes.byref(s)))
        return s.as_dict()

    # ---- beams ----
    def set_beams(self, start, end, radius, power):
        """Host arrays (numpy): copies to the GPU and builds the BVH."""
        start, end, radius, power = (_f32(x) for x in (start, end, radius, power))
        n = radius.shape[0]
        assert start.shape == (n, 3) and end.shape == (n, 3) and power.shape == (n, 3)
        self._check(self.lib.bre_set_beams(self.h, n, _ptr(start), _ptr(end), _ptr(radius), _ptr(power)))

    def set_beams_device(self, start, end, radius, power):
        """Device tensors (torch, float32, contiguous)."""
        n = radius.shape[0]
        for t in (start, end, radius, power):
            assert t.is_cuda and t.is_contiguous() and str(t.dtype) == "torch.float32"
        self._keep = [start, end, radius, power]
        self._check(self.lib.bre_set_beams_device(self.h, n, _ptr(start), _ptr(end), _ptr(radius), _ptr(power)))

    # ---- photon pass ----
    def trace_photons(self, scene, n_photons: int, iteration: int = 0, max_depth: int = 5,
                      radius: float = 0.01) -> int:
        """Photon pass on the GPU (photonbeam.cpp:362-438): traces, keeps and builds the beams.
        `scene` is a scene.Scene (ctypes).  Returns the number of beams."""
        nb = ctypes.c_int64(0)
        self._check(self.lib.bre_trace_photons(self.h, ctypes.addressof(scene), int(n_photons), int(iteration),
                                               int(max_depth), float(radius), ctypes.byref(nb)))
        return nb.value

    def get_beams(self):
        """Copy the current beam set back: dict start/end (n,3), radius (n,), power (n,3)."""
        nb = ctypes.c_int64(0)
        self._check(self.lib.bre_get_beams(self.h, 0, None, None, None, None, ctypes.byref(nb)))
        n = nb.value
        out = {"start": np.zeros((n, 3), np.float32), "end": np.zeros((n, 3), np.float32),
               "radius": np.zeros(n, np.float32), "power": np.zeros((n, 3), np.float32)}
        self._check(self.lib.bre_get_beams(self.h, n, _ptr(out["start"]), _ptr(out["end"]), _ptr(out["radius"]),
                                           _ptr(out["power"]), ctypes.byref(nb)))
        return out

    # ---- camera pass ----
    def camera_pass(self, scene, width: int, height: int, iteration: int = 0, max_depth: int = 5,
                    render_surfaces: bool = True, render_media: bool = True, surface=None) -> int:
        """Camera pass on the GPU (photonbeam.cpp:444-555).  `surface`: optional torch float32
        CUDA tensor (W*H, 3) receiving += the surface radiance.  Returns the segment count."""
        n = ctypes.c_int64(0)
        self._film(surface, int(width) * int(height), "camera_pass surface")
        self._check(self.lib.bre_camera_pass(self.h, ctypes.addressof(scene), int(width), int(height),
                                             int(iteration), int(max_depth), int(render_surfaces),
                                             int(render_media), _ptr(surface), ctypes.byref(n)))
        self._cam_npix = int(width) * int(height)
        return n.value

    def gather_camera(self, R: float, accum):
        """Gather the last camera pass's segments into `accum` (torch CUDA tensor (W*H, 3))."""
        self._film(accum, self._cam_npix, "gather_camera accum")
        self._check(self.lib.bre_gather_camera(self.h, float(R), _ptr(accum)))

    def gather_camera_segments(self, R: float, accum=None, seg_rgb=None, counts=None):
        """bre_gather_camera with per-segment outputs (torch CUDA tensors, camera-pass order):
        seg_rgb (n, 3) float32, counts (n, 2) int32 ({C or -1, contributions})."""
        self._film(accum, self._cam_npix, "gather_camera_segments accum")
        self._check(self.lib.bre_gather_camera_segments(self.h, float(R), _ptr(accum), _ptr(seg_rgb), _ptr(counts)))

    def get_segments(self):
        n = ctypes.c_int64(0)
        self._check(self.lib.bre_get_segments(self.h, 0, None, None, None, None, None, None, ctypes.byref(n)))
        k = n.value
        out = {"o": np.zeros((k, 3), np.float32), "p": np.zeros((k, 3), np.float32), "d": np.zeros((k, 3), np.float32),
               "tmax": np.zeros(k, np.float32), "pixel": np.zeros(k, np.int32), "depth": np.zeros(k, np.int32)}
        self._check(self.lib.bre_get_segments(self.h, k, _ptr(out["o"]), _ptr(out["p"]), _ptr(out["d"]),
                                              _ptr(out["tmax"]), _ptr(out["pixel"]), _ptr(out["depth"]),
                                              ctypes.byref(n)))
        return out

    # ---- the integrator ----
    def render_iteration(self, scene, params, iteration: int, ld):
        self._film(ld, int(params.width) * int(params.height), "render_iteration ld")
        self._check(self.lib.bre_render_iteration(self.h, ctypes.addressof(scene), ctypes.addressof(params),
                                                  int(iteration), _ptr(ld)))

    def render(self, scene, params):
        """Whole PhotonBeamIntegrator::Render; returns the (H, W, 3) float32 image Ld / end_iteration."""
        img = np.zeros((params.height, params.width, 3), np.float32)
        self._check(self.lib.bre_render(self.h, ctypes.addressof(scene), ctypes.addressof(params), _ptr(img)))
        return img

    # ---- gather ----
    def gather(self, o, p, d, tmax, pixel=None, R=0.01, npix=0, accum=None, seg_rgb=True, counts=False):
        """Host arrays.  Returns dict with 'seg_rgb' (nseg,3) and optionally 'counts' (nseg,2);
        `accum` (npix,3) float32 is updated in place when given."""
        o, p, d, tmax = (_f32(x) for x in (o, p, d, tmax))
        n = tmax.shape[0]
        pix = None if pixel is None else np.ascontiguousarray(pixel, dtype=np.int32)
        out = np.zeros((n, 3), np.float32) if seg_rgb else None
        cnt = np.zeros((n, 2), np.int32) if counts else None
        if accum is not None:
            assert accum.dtype == np.float32 and accum.flags.c_contiguous
        self._check(self.lib.bre_gather(self.h, n, _ptr(o), _ptr(p), _ptr(d), _ptr(tmax), _ptr(pix), float(R),
                                        int(npix), _ptr(accum), _ptr(out), _ptr(cnt)))
        res = {}
        if out is not None:
            res["seg_rgb"] = out
        if cnt is not None:
            res["counts"] = cnt
        return res

    def gather_device(self, o, p, d, tmax, pixel, R, npix, accum=None, seg_rgb=None, counts=None):
        """Device tensors; asynchronous on the context stream."""
        n = tmax.shape[0]
        self._film(accum, npix, "gather_device accum")
        self._check(self.lib.bre_gather_device(self.h, n, _ptr(o), _ptr(p), _ptr(d), _ptr(tmax), _ptr(pixel),
                                               float(R), int(npix), _ptr(accum), _ptr(seg_rgb), _ptr(counts)))

    def device_check(self, kind: int, x, aux=None):
        """bre_device_check: libbre's device copies of NextFloatUp/Down (kinds 0/1), the exact
        stage's square root next to sqrtf (2), FindInterval over aux (3) and the shared-reciprocal
        division next to x / aux[0] (4), the passes' expf / logf / sinf / cosf (9).  Returns float32
        [n], [n, 2] (kinds 2, 4) or [n, 4] (kind 9)."""
        x = np.ascontiguousarray(x, dtype=np.float32)
        n = x.shape[0]
        w = 4 if kind == 9 else 2 if kind in (2, 4) else 1
        y = np.zeros((n, w) if w > 1 else n, np.float32)
        a = None if aux is None else np.ascontiguousarray(aux, dtype=np.float32)
        self._check(self.lib.bre_device_check(self.h, kind, n, _ptr(x), 0 if a is None else a.shape[0],
                                              None if a is None else _ptr(a), _ptr(y)))
        return y

    def slot_sort(self, keys, begin_bit: int = 0, end_bit: int | None = None):
        """bre_device_check kinds 6 / 8: the pass chain's stable radix sort (bre_slot.hip) of uint64 or
        uint32 keys; returns (sorted keys, the permutation)."""
        k = np.ascontiguousarray(keys)
        kb = k.dtype.itemsize
        if k.dtype not in (np.uint64, np.uint32):
            raise ValueError("slot_sort: uint64 or uint32 keys")
        m = k.shape[0]
        end_bit = 8 * kb if end_bit is None else end_bit
        x = k.view(np.uint32)
        y = np.zeros(m * (kb + 4) // 4 + 1, np.uint32)
        a = np.array([begin_bit, end_bit], np.float32)
        self._check(self.lib.bre_device_check(self.h, 6 if kb == 8 else 8, x.shape[0], _ptr(x), 2, _ptr(a), _ptr(y)))
        sk = y[: m * kb // 4].view(k.dtype).copy()
        perm = y[m * kb // 4: m * kb // 4 + m].view(np.int32).copy()
        return sk, perm

    def slot_scan(self, values):
        """bre_device_check kind 7: the pass chain's exclusive scan (bre_slot.hip) of int32 values;
        returns int64 [n + 1] (the total last)."""
        v = np.ascontiguousarray(values, dtype=np.int32)
        y = np.zeros(v.shape[0] + 1, np.int64)
        self._check(self.lib.bre_device_check(self.h, 7, v.shape[0], _ptr(v), 0, None, _ptr(y)))
        return y

    def work_roots(self, children, nleaf, S: int):
        """bre_device_check kind 5: the tile kernel's S work roots (k_roots) of a binary tree given as
        children [(c0, c1)] (>= 0 node, < 0 leaf ~k, EMPTY_CHILD none) and nleaf per node, node 0 the
        root.  Returns the roots, largest first."""
        m = len(children)
        rec = np.zeros((m, 16), np.int32)
        for i, (c0, c1) in enumerate(children):
            rec[i, 12], rec[i, 13], rec[i, 14], rec[i, 15] = c0, c1, -1, nleaf[i]
        x = rec.view(np.float32).ravel()
        y = np.zeros(S + 1, np.int32)
        a = np.array([S], np.float32)
        self._check(self.lib.bre_device_check(self.h, 5, x.shape[0], _ptr(x), 1, _ptr(a), _ptr(y)))
        return [int(v) for v in y[:int(y[S])]]

    def close(self):
        if getattr(self, "h", None):
            self.lib.bre_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def _ctx_array(ctxs):
    arr = (ctypes.c_void_p * len(ctxs))(*[c.h.value for c in ctxs])
    return arr


def _check_group(ctxs, st):
    if st != BRE_OK:
        raise BreError(st, ctxs[0].lib.bre_last_error(ctxs[0].h).decode())


def set_beams_sharded(ctxs, start, end, radius, power):
    """bre_set_beams_sharded: the same beam set (host arrays) built on every context, in parallel."""
    start, end, radius, power = (_f32(x) for x in (start, end, radius, power))
    n = radius.shape[0]
    _check_group(ctxs, ctxs[0].lib.bre_set_beams_sharded(_ctx_array(ctxs), len(ctxs), n, _ptr(start), _ptr(end),
                                                         _ptr(radius), _ptr(power)))


def gather_sharded(ctxs, o, p, d, tmax, pixel=None, R=0.01, npix=0, accum=None, seg_rgb=True, counts=False):
    """bre_gather_sharded over BeamGather contexts (one per GPU): host arrays, as BeamGather.gather."""
    o, p, d, tmax = (_f32(x) for x in (o, p, d, tmax))
    n = tmax.shape[0]
    pix = None if pixel is None else np.ascontiguousarray(pixel, dtype=np.int32)
    out = np.zeros((n, 3), np.float32) if seg_rgb else None
    cnt = np.zeros((n, 2), np.int32) if counts else None
    if accum is not None:
        assert accum.dtype == np.float32 and accum.flags.c_contiguous
    _check_group(ctxs, ctxs[0].lib.bre_gather_sharded(_ctx_array(ctxs), len(ctxs), n, _ptr(o), _ptr(p), _ptr(d),
                                                      _ptr(tmax), _ptr(pix), float(R), int(npix), _ptr(accum),
                                                      _ptr(out), _ptr(cnt)))
    res = {}
    if out is not None:
        res["seg_rgb"] = out
    if cnt is not None:
        res["counts"] = cnt
    return res


def shard_segments(n_segments: int, rank: int, count: int, chunk: int = 1) -> int:
    """How many camera segments shard `rank` of `count` gathers in packet mode (libbre)."""
    return int(load_library().bre_shard_segments(int(n_segments), int(rank), int(count), int(chunk)))


def shard_packet_index(n_segments: int, rank: int, count: int, chunk: int = 1):
    """The segment indices (in the gathered order) of shard `rank`'s packets -- chunks of `chunk`
    consecutive packets, chunk c to shard c mod count: the host view of libbre's packet pick, for tests
    and CPU rehearsals."""
    import numpy as np
    npk = (int(n_segments) + 63) // 64
    nch = (npk + chunk - 1) // chunk
    pk = (np.arange(rank, nch, count, dtype=np.int64)[:, None] * chunk + np.arange(chunk)[None, :]).ravel()
    pk = pk[pk < npk]
    idx = (pk[:, None] * 64 + np.arange(64)[None, :]).ravel()
    return idx[idx < n_segments]


def beam_radius_at(initial_radius: float, alpha: float, iteration: int) -> float:
    """currentBeamRadius at `iteration` (photonbeam.cpp:354-356, 562), via libbre."""
    return float(load_library().bre_beam_radius_at(initial_radius, alpha, iteration))
