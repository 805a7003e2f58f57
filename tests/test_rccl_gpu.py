"""The framebuffer collectives over RCCL on the GPU ("next round" item 4).

The north star's multi-GPU path ends in one RCCL collective per written image
(photonbeam.cpp:565-584 after the split of :444-557 over ranks): packet shards sum-reduce their
partial films (dist.reduce on device tensors), tile shards gather their owned-pixel bands
(dist.gather).  Until round 4 both had run only over gloo.  Here a world-size-1 "nccl" (= RCCL on
ROCm) process group is initialised in the test process itself (env:// on a free 127.0.0.1 port; no
exec, no relaunch), a real C2-style film is rendered by libbre on cuda:0, and both collectives run on
it: the root's film after ShardedFrame.gather_to_root must be bit-equal to the local film, in packet
mode and in tile mode, and the gathered band must be the local band bit for bit.  The 8-GPU job of
the driver then is not the first execution of this code."""
import importlib
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture(scope="module")
def nccl_group():
    import torch
    import torch.distributed as dist

    assert not dist.is_initialized()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    os.environ["RANK"] = "0"
    os.environ["WORLD_SIZE"] = "1"
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="env://", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    yield dist
    dist.destroy_process_group()


def _render_film(bre, scene_mod, frame, W, H):
    import torch

    scene = scene_mod.cornell_scene(0.05, 0.5, 0.0)
    R = bre.beam_radius_at(0.01, 0.5, 0)
    with bre.BeamGather(0) as g:
        g.set_shard(0, 1, frame.block, frame.packets)
        g.trace_photons(scene, 100_000, 0, 5, R)
        g.camera_pass(scene, W, H, 0, 5, True, True, frame.accum)
        g.gather_camera(R, frame.accum)
        g.synchronize()
    torch.cuda.synchronize()


@pytest.mark.parametrize("packets", [True, False])
def test_rccl_framebuffer_collective_world1(bre, scene_mod_gpu, nccl_group, packets):
    import torch

    dmod = importlib.import_module("beam-radiance-estimate-pbrt_amd.dist")
    W = H = 128
    frame = dmod.ShardedFrame(W, H, 0, 1, device=torch.device("cuda", 0), packets=packets)
    _render_film(bre, scene_mod_gpu, frame, W, H)
    local = frame.accum.clone()
    assert float(local.abs().sum()) > 0
    if not packets:
        parts = frame.gather_bands(0)
        assert len(parts) == 1 and parts[0].is_cuda
        assert torch.equal(parts[0], frame.band())
    out = frame.gather_to_root(0)
    torch.cuda.synchronize()
    assert out.is_cuda
    assert np.array_equal(out.cpu().numpy().view(np.uint32), local.cpu().numpy().view(np.uint32))
