"""Python view of libbre_host.so (include/bre_pbrt.h): the .pbrt scene front end, the
photon-beam integrator's Render on the GPU, and the film / PFM output.

    sc = pbrt.parse_file("scenes/cornell_fog_c2.pbrt")   # pbrtParseFile (api.cpp, pbrtparse.y)
    sc.scene, sc.params, sc.film                          # bre_scene, bre_render_params, film
    img = sc.render(device=0, write_files=False)          # WorldEnd -> PhotonBeamIntegrator::Render

The parser, integrator mirror and film code are C++ (host/pbrt_scene.cpp, host/photonbeam_gpu.cpp);
this module only declares their C signatures.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import load_library
from .scene import RenderParams, Scene

HERE = os.path.dirname(os.path.abspath(__file__))
HOST_LIB_PATH = os.path.join(HERE, "libbre_host.so")
CLI_PATH = os.path.join(HERE, "host", "bre_pbrt")

EXPORTS = ["bre_pbrt_parse_file", "bre_pbrt_parse_string", "bre_pbrt_free", "bre_pbrt_messages",
           "bre_pbrt_get_scene", "bre_pbrt_get_render_params", "bre_pbrt_get_film", "bre_pbrt_render",
           "bre_film_finalize", "bre_write_pfm", "bre_read_pfm"]

_HOST = None


def load_host_library(path: str = HOST_LIB_PATH) -> ctypes.CDLL:
    global _HOST
    if _HOST is not None:
        return _HOST
    load_library()  # libbre.so first (torch's HIP runtime ordering, see load_library)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not found: build it with `make -C {HERE}/host`")
    lib = ctypes.CDLL(path)
    P, I64, I32, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float
    lib.bre_pbrt_parse_file.argtypes = [ctypes.c_char_p, ctypes.POINTER(P)]
    lib.bre_pbrt_parse_string.argtypes = [ctypes.c_char_p, ctypes.POINTER(P)]
    lib.bre_pbrt_free.argtypes = [P]
    lib.bre_pbrt_free.restype = None
    lib.bre_pbrt_messages.argtypes = [P, ctypes.POINTER(I32), ctypes.POINTER(I32)]
    lib.bre_pbrt_messages.restype = ctypes.c_char_p
    lib.bre_pbrt_get_scene.argtypes = [P, P]
    lib.bre_pbrt_get_render_params.argtypes = [P, I32, P, ctypes.POINTER(I32)]
    lib.bre_pbrt_get_film.argtypes = [P, ctypes.POINTER(I32), ctypes.POINTER(I32), ctypes.POINTER(F),
                                      ctypes.c_char_p, I32]
    lib.bre_pbrt_render.argtypes = [P, I32, I32, ctypes.c_char_p, I32, P]
    lib.bre_film_finalize.argtypes = [I64, P, F, P]
    lib.bre_write_pfm.argtypes = [ctypes.c_char_p, P, I32, I32]
    lib.bre_read_pfm.argtypes = [ctypes.c_char_p, P, I64, ctypes.POINTER(I32), ctypes.POINTER(I32)]
    for n in EXPORTS:
        if n not in ("bre_pbrt_free", "bre_pbrt_messages"):
            getattr(lib, n).restype = I32
    _HOST = lib
    return lib


class PbrtError(RuntimeError):
    pass


class PbrtScene:
    """A parsed scene (owns the C handle)."""

    def __init__(self, handle, ok: bool, quick: bool = False):
        self._lib = load_host_library()
        self._h = handle
        ne, nw = ctypes.c_int32(), ctypes.c_int32()
        self.messages = self._lib.bre_pbrt_messages(self._h, ctypes.byref(ne), ctypes.byref(nw)).decode()
        self.n_errors, self.n_warnings = ne.value, nw.value
        self.ok = ok
        self.quick = quick
        if not ok:
            return
        self.scene = Scene()
        assert self._lib.bre_pbrt_get_scene(self._h, ctypes.byref(self.scene)) == 0
        self.params = RenderParams()
        wf = ctypes.c_int32()
        assert self._lib.bre_pbrt_get_render_params(self._h, int(quick), ctypes.byref(self.params), ctypes.byref(wf)) == 0
        self.write_frequency = wf.value
        w, h, sc = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_float()
        buf = ctypes.create_string_buffer(4096)
        assert self._lib.bre_pbrt_get_film(self._h, ctypes.byref(w), ctypes.byref(h), ctypes.byref(sc), buf, 4096) == 0
        self.film = dict(xres=w.value, yres=h.value, scale=sc.value, filename=buf.value.decode())

    def render(self, device: int = 0, outfile: str | None = None, write_files: bool = True) -> np.ndarray:
        """PhotonBeamIntegrator::Render on GPU `device`; returns the last film image (H, W, 3)."""
        if not self.ok:
            raise PbrtError(self.messages)
        img = np.zeros((self.film["yres"], self.film["xres"], 3), np.float32)
        st = self._lib.bre_pbrt_render(self._h, int(device), int(self.quick),
                                       outfile.encode() if outfile else None, int(write_files),
                                       img.ctypes.data_as(ctypes.c_void_p))
        if st != 0:
            raise PbrtError(f"bre_pbrt_render failed with status {st}")
        return img

    def close(self):
        if self._h:
            self._lib.bre_pbrt_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _parse(fn, arg: bytes, quick: bool) -> PbrtScene:
    lib = load_host_library()
    h = ctypes.c_void_p()
    st = getattr(lib, fn)(arg, ctypes.byref(h))
    return PbrtScene(h, st == 0, quick)


def parse_file(path: str, quick: bool = False) -> PbrtScene:
    return _parse("bre_pbrt_parse_file", os.fsencode(path), quick)


def parse_string(text: str, quick: bool = False) -> PbrtScene:
    return _parse("bre_pbrt_parse_string", text.encode(), quick)


def film_finalize(L: np.ndarray, scale: float = 1.0) -> np.ndarray:
    """Film::SetImage(L) + Film::WriteImage's per-pixel conversion (film.cpp:132-210)."""
    L = np.ascontiguousarray(L, dtype=np.float32)
    out = np.empty_like(L)
    st = load_host_library().bre_film_finalize(L.size // 3, L.ctypes.data_as(ctypes.c_void_p), float(scale),
                                               out.ctypes.data_as(ctypes.c_void_p))
    if st != 0:
        raise PbrtError(f"bre_film_finalize failed with status {st}")
    return out


def write_pfm(path: str, rgb: np.ndarray) -> None:
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = rgb.shape[:2]
    if load_host_library().bre_write_pfm(os.fsencode(path), rgb.ctypes.data_as(ctypes.c_void_p), w, h) != 0:
        raise PbrtError(f"cannot write {path}")


def read_pfm(path: str) -> np.ndarray:
    lib = load_host_library()
    w, h = ctypes.c_int32(), ctypes.c_int32()
    if lib.bre_read_pfm(os.fsencode(path), None, 0, ctypes.byref(w), ctypes.byref(h)) != 0:
        raise PbrtError(f"cannot read {path}")
    out = np.empty((h.value, w.value, 3), np.float32)
    lib.bre_read_pfm(os.fsencode(path), out.ctypes.data_as(ctypes.c_void_p), out.size, ctypes.byref(w), ctypes.byref(h))
    return out
