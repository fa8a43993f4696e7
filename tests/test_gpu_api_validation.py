"""
GPU tests of the host-side argument checks of the device drop-in
(`gridder.device_ms2dirty`, `accumulate.GridAccumulator.dirty`): the library
writes npix_x * npix_y doubles through `out` and one double through
`sum_weights`, so a wrong dtype, shape, layout or device must raise
ValueError before the call instead of corrupting HBM.
"""
import numpy as np
import pytest

from ska_sdp_cip_amd import gridder, synthetic as syn

pytestmark = pytest.mark.gpu


def _inputs(npix=64):
    import torch

    uvw = syn.uvw_tracks(200, 8, array_radius_m=500.0, seed=2)
    f = syn.channel_frequencies(4)
    rng = np.random.default_rng(0)
    vis = (rng.standard_normal((uvw.shape[0], 4)) + 1j).astype(np.complex64)
    w = np.ones(vis.shape, np.float32)
    px = syn.pixel_size_for_grid(uvw, f, npix)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    return (t(uvw), t(f), t(vis), t(w), npix, npix, px, px)


@pytest.mark.parametrize("bad", ["f32", "shape", "strided", "cpu"])
def test_out_is_validated(gpu_device, bad):
    import torch

    args = _inputs()
    out = {
        "f32": lambda: torch.zeros((64, 64), dtype=torch.float32, device="cuda"),
        "shape": lambda: torch.zeros((32, 64), dtype=torch.float64, device="cuda"),
        "strided": lambda: torch.zeros((64, 128), dtype=torch.float64, device="cuda")[:, ::2],
        "cpu": lambda: torch.zeros((64, 64), dtype=torch.float64),
    }[bad]()
    with pytest.raises(ValueError):
        gridder.device_ms2dirty(*args, support=8, out=out)


@pytest.mark.parametrize("bad", ["f32", "two", "cpu"])
def test_sum_weights_is_validated(gpu_device, bad):
    import torch

    args = _inputs()
    sw = {
        "f32": lambda: torch.zeros(1, dtype=torch.float32, device="cuda"),
        "two": lambda: torch.zeros(2, dtype=torch.float64, device="cuda"),
        "cpu": lambda: torch.zeros(1, dtype=torch.float64),
    }[bad]()
    with pytest.raises(ValueError):
        gridder.device_ms2dirty(*args, support=8, sum_weights=sw)


def test_valid_out_and_sum_weights_are_used(gpu_device):
    import torch

    args = _inputs()
    out = torch.full((64, 64), 7.0, dtype=torch.float64, device="cuda")
    sw = torch.zeros(1, dtype=torch.float64, device="cuda")
    res, _ = gridder.device_ms2dirty(*args, support=8, out=out, sum_weights=sw)
    torch.cuda.synchronize()
    assert res.data_ptr() == out.data_ptr()
    assert float(sw.item()) == float(args[3].double().sum().item())
    assert not torch.any(out == 7.0)


def test_workspace_release_and_thread_exit(gpu_device):
    """cip_release_workspace frees the calling thread's workspace (a later call
    rebuilds it); workspaces of a worker thread are freed when it exits."""
    import threading

    import torch

    from ska_sdp_cip_amd import _lib

    args = _inputs(1024)  # 2048^2 grid: 64 MiB per workspace
    ref, _ = gridder.device_ms2dirty(*args, support=8)
    ref = ref.clone()
    _lib.check(_lib.lib().cip_release_workspace())
    again, _ = gridder.device_ms2dirty(*args, support=8)
    assert torch.equal(ref, again)
    results = []

    def worker():
        d, _ = gridder.device_ms2dirty(*args, support=8)
        torch.cuda.synchronize()
        results.append(d.cpu())

    def run_thread():
        th = threading.Thread(target=worker)
        th.start()
        th.join()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()

    # the first worker thread settles the runtime's per-thread state and
    # torch's allocator; free memory after it is the steady state
    run_thread()
    free1 = torch.cuda.mem_get_info()[0]
    for _ in range(3):
        run_thread()
    assert all(torch.equal(ref.cpu(), r) for r in results)
    # exited threads hold no workspace: each one would keep a 64 MiB grid and
    # a 32 MiB FFT intermediate, so three leaked workspaces lose > 280 MiB
    assert torch.cuda.mem_get_info()[0] > free1 - 32 * 1024 * 1024


@pytest.mark.parametrize("wstack,resident", [(False, True), (True, True), (False, False)])
def test_async_call_matches_synchronous(gpu_device, wstack, resident):
    """synchronize=False (CIP_ASYNC) queues the whole invert and returns; with
    resident_inputs=True (CIP_PIPELINE) its planner runs on the workspace's plan
    stream beside the previous calls' scatter and FFT. In stream order each
    image and weight sum equal the synchronous call's, also for back-to-back
    pipelined calls (alternating planner buffers)."""
    import torch

    a = _inputs(512)
    # a second resident input set (other visibilities and weights): calls
    # alternate between the two, so consecutive plans, dirty-tile masks and
    # weight sums differ
    b = (a[0], a[1], a[2] * (0.5 - 2.0j), a[3] * 0.25 + 1.0) + a[4:]
    sets = [a, b]
    refs = []
    for args in sets:
        ref, _ = gridder.device_ms2dirty(*args, support=8, normalise=True, do_wstacking=wstack)
        refs.append(ref.clone())
    outs = []
    for k in range(6):
        out = torch.empty_like(refs[0])
        sw = torch.empty(1, dtype=torch.float64, device=out.device)
        gridder.device_ms2dirty(*sets[k % 2], support=8, normalise=True, out=out, sum_weights=sw,
                                synchronize=False, resident_inputs=resident, do_wstacking=wstack)
        outs.append((out, sw))
    torch.cuda.synchronize()
    for k, (out, sw) in enumerate(outs):
        assert torch.equal(out, refs[k % 2])
        assert float(sw.item()) == float(sets[k % 2][3].double().sum().item())


def test_pipelined_calls_interleaved_with_other_calls(gpu_device):
    """Pipelined calls (planner on the plan streams) interleaved with calls of
    another kind - synchronous, asynchronous without resident inputs,
    pipelined w-stacking - that also use the workspace grid and planner
    buffers. Every image equals its synchronous reference."""
    import torch

    a = _inputs(512)
    b = (a[0], a[1], a[2] * (0.5 - 2.0j), a[3] * 0.25 + 1.0) + a[4:]
    ref = {}
    for name, args in (("a", a), ("b", b)):
        for ws in (False, True):
            img, _ = gridder.device_ms2dirty(*args, support=8, normalise=True, do_wstacking=ws)
            ref[name, ws] = img.clone()
    seq = [("a", "pipe", False), ("b", "pipe", False), ("a", "sync", False), ("b", "pipe", False),
           ("a", "async", False), ("b", "pipe", False), ("a", "pipe", True), ("b", "pipe", False),
           ("a", "pipe", False), ("b", "pipe", True), ("a", "pipe", False)]
    outs = []
    for name, mode, ws in seq:
        out = torch.empty_like(ref["a", False])
        gridder.device_ms2dirty(*(a if name == "a" else b), support=8, normalise=True, out=out,
                                synchronize=mode == "sync", resident_inputs=mode == "pipe", do_wstacking=ws)
        outs.append(out)
    torch.cuda.synchronize()
    for (name, mode, ws), out in zip(seq, outs):
        assert torch.equal(out, ref[name, ws]), (name, mode, ws)


def test_async_call_sees_inputs_written_on_the_stream(gpu_device):
    """Without resident_inputs, an asynchronous call starts in stream order: a
    kernel that rewrites the visibilities between two calls is seen by the
    second call (its planner must not run ahead of the stream)."""
    import torch

    uvw, f, vis, w, nx, ny, px, py = _inputs(512)
    vis2 = vis * 3.0
    ref1, _ = gridder.device_ms2dirty(uvw, f, vis, w, nx, ny, px, py, support=8)
    ref1 = ref1.clone()
    ref2, _ = gridder.device_ms2dirty(uvw, f, vis2, w, nx, ny, px, py, support=8)
    ref2 = ref2.clone()
    torch.cuda.synchronize()
    work = vis.clone()
    outs = [torch.empty_like(ref1) for _ in range(4)]
    for k, out in enumerate(outs):
        # stream order: the copy runs after the previous call's work is queued
        work.copy_(vis if k % 2 == 0 else vis2)
        gridder.device_ms2dirty(uvw, f, work, w, nx, ny, px, py, support=8, out=out, synchronize=False)
    torch.cuda.synchronize()
    for k, out in enumerate(outs):
        assert torch.equal(out, ref1 if k % 2 == 0 else ref2)


def test_resident_inputs_needs_async(gpu_device):
    with pytest.raises(ValueError):
        gridder.device_ms2dirty(*_inputs(), support=8, synchronize=True, resident_inputs=True)
