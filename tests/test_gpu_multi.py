"""Several GPUs behind the C-ABI (rt_multi, rt_comm), on the one
GPU of the test box: a device list may name cuda:0 more than once, which
RCCL refuses, so those runs take the peer-copy transport; a one-device list
runs the RCCL transport (grouped send/recv to itself).  Every gathered frame
must be bit-identical to one device's rt_trace of the whole frame (and to the
oracle): samples are never split across devices, so no bit may move."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def single(rt, torch, scene, cam, W, H, frames, B, simd=True, prev_count=0, prev=None):
    dev = rt.Device(0)
    try:
        dev.upload_scene(scene)
        if prev is None:
            prev = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        cur = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        rays = torch.zeros(1, dtype=torch.int64, device="cuda")
        dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(), rays_ptr=rays.data_ptr(),
                  prev_count=prev_count, frames=frames, max_bounce=B, simd=simd, band_rows=8,
                  stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        return prev, cur, int(rays.item())
    finally:
        dev.close()


def multi_render(rt, torch, m, cam, W, H, frames, B, simd=True, prev_count=0, accum_zero=False, band_rows=8):
    cur = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    prev = torch.full((W * H, 4), float("nan"), dtype=torch.float32, device="cuda")
    rays = torch.zeros(1, dtype=torch.int64, device="cuda")
    m.trace(cam, width=W, height=H, cur_ptr=cur.data_ptr(), prev_ptr=prev.data_ptr(), rays_ptr=rays.data_ptr(),
            prev_count=prev_count, frames=frames, max_bounce=B, simd=simd, band_rows=band_rows,
            accum_zero=accum_zero, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return prev, cur, int(rays.item())


def same(a, b):
    assert a[2] == b[2], (a[2], b[2])
    assert torch_equal_bits(a[0], b[0]), "running mean differs"
    assert torch_equal_bits(a[1], b[1]), "RGBA8 differs"


def torch_equal_bits(x, y):
    return np.array_equal(x.cpu().numpy().view(np.uint32), y.cpu().numpy().view(np.uint32))


@pytest.mark.parametrize("devices,transport", [([0], "rccl"), ([0], "peer"), ([0, 0], "auto"), ([0, 0, 0], "auto"),
                                               ([0] * 8, "auto")])
def test_multi_equals_single_device(rt, orc, torch_cuda, devices, transport):
    torch = torch_cuda
    t = {"rccl": rt.RT_MULTI_RCCL, "peer": rt.RT_MULTI_PEER, "auto": rt.RT_MULTI_AUTO}[transport]
    s = rt.scene_prefix(rt.scene_builtin(1), 64)
    W, H, S, B = 200, 150, 4, 8  # 19 bands of 8 rows, the last one partial
    cam = rt.camera_setup(s, W, H)
    ref = single(rt, torch, s, cam, W, H, S, B)
    m = rt.Multi(devices, t)
    try:
        info = m.info()
        assert info["DeviceCount"] == len(devices)
        assert info["Transport"] == (rt.RT_MULTI_RCCL if transport == "rccl" else rt.RT_MULTI_PEER)
        m.upload_scene(s)
        got = multi_render(rt, torch, m, cam, W, H, S, B, accum_zero=True)
        same(got, ref)
        o = orc.scene_builtin(1).prefix(64)
        op, oc, orays = orc.render(o, orc.camera(o, W, H), W, H, frames=S, max_bounce=B)
        assert orays == got[2] and np.array_equal(got[1].cpu().numpy().view(np.uint32), oc)
    finally:
        m.close()


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_multi_progressive_running_mean_stays_on_the_devices(rt, torch_cuda, devices):
    """Frames 0-2 then 3-7 (PreviousRayCount 3, the running mean resident on
    the devices) equal one 8-frame single-device launch; scalar rules too."""
    torch = torch_cuda
    s = rt.scene_builtin(0)
    W, H, B = 96, 72, 5
    cam = rt.camera_setup(s, W, H)
    for simd in (True, False):
        ref = single(rt, torch, s, cam, W, H, 8, B, simd=simd)
        m = rt.Multi(devices)
        try:
            m.upload_scene(s)
            a = multi_render(rt, torch, m, cam, W, H, 3, B, simd=simd)
            b = multi_render(rt, torch, m, cam, W, H, 5, B, simd=simd, prev_count=3)
            assert a[2] + b[2] == ref[2]
            same((b[0], b[1], ref[2]), ref)
        finally:
            m.close()


def test_multi_rejects_continuation_without_a_resident_mean(rt, torch_cuda):
    torch = torch_cuda
    s = rt.scene_prefix(rt.scene_builtin(1), 16)
    cam = rt.camera_setup(s, 64, 48)
    m = rt.Multi([0, 0])
    try:
        m.upload_scene(s)
        with pytest.raises(rt.RtError):
            multi_render(rt, torch, m, cam, 64, 48, 2, 4, prev_count=2)
        multi_render(rt, torch, m, cam, 64, 48, 2, 4)
        with pytest.raises(rt.RtError):  # geometry changed: the resident mean is gone
            multi_render(rt, torch, m, cam, 64, 40, 2, 4, prev_count=2)
    finally:
        m.close()


def test_multi_rejects_a_wrong_previous_ray_count(rt, torch_cuda):
    """The resident means hold the frames folded so far; a continuation that
    claims another count would blend with the wrong weights."""
    torch = torch_cuda
    s = rt.scene_prefix(rt.scene_builtin(1), 16)
    cam = rt.camera_setup(s, 64, 48)
    m = rt.Multi([0, 0])
    try:
        m.upload_scene(s)
        multi_render(rt, torch, m, cam, 64, 48, 2, 4)
        with pytest.raises(rt.RtError, match="holds 2 frames"):
            multi_render(rt, torch, m, cam, 64, 48, 2, 4, prev_count=3)
        multi_render(rt, torch, m, cam, 64, 48, 3, 4, prev_count=2)
        multi_render(rt, torch, m, cam, 64, 48, 1, 4, prev_count=5)
    finally:
        m.close()


@pytest.mark.parametrize("devices", [[0, 0, 0], [0] * 8])
def test_multi_calls_back_to_back_overlap_gather_and_trace(rt, orc, torch_cuda, devices):
    """Calls enqueued back to back with no host synchronisation: each device
    alternates between two band-image slots, so call k's gather overlaps call
    k+1's traces and a slot is reused only after the gather two calls back.
    Five calls with three cameras (new cull keys included) into five frames,
    each bit-identical to one device's render; per-device trace times exist."""
    torch = torch_cuda
    s = rt.scene_prefix(rt.scene_builtin(1), 64)
    W, H, S, B = 200, 150, 4, 8
    views = [(None, None), (6.0, 0.7), (None, None), (2.0, -1.1), (None, None)]
    cams = [rt.camera_setup(s, W, H, distance=d, x_angle=a) for d, a in views]
    refs = [single(rt, torch, s, c, W, H, S, B) for c in cams[:2]] + [None] + \
           [single(rt, torch, s, cams[3], W, H, S, B)] + [None]
    refs[2] = refs[4] = refs[0]
    m = rt.Multi(devices)
    try:
        m.upload_scene(s)
        outs = []
        st = torch.cuda.current_stream().cuda_stream
        for cam in cams:
            cur = torch.zeros(W * H, dtype=torch.int32, device="cuda")
            rays = torch.zeros(1, dtype=torch.int64, device="cuda")
            m.trace(cam, width=W, height=H, cur_ptr=cur.data_ptr(), rays_ptr=rays.data_ptr(), frames=S,
                    max_bounce=B, band_rows=8, accum_zero=True, stream=st)
            outs.append((cur, rays))
        ms = m.last_trace_ms(len(devices))
        torch.cuda.synchronize()
    finally:
        m.close()
    assert len(ms) == len(devices) and all(v >= 0.0 for v in ms)
    for (cur, rays), ref in zip(outs, refs):
        assert int(rays.item()) == ref[2]
        assert torch_equal_bits(cur, ref[1]), "RGBA8 differs"


def test_multi_rccl_refuses_a_device_listed_twice(rt, torch_cuda):
    with pytest.raises(rt.RtError, match="RCCL"):
        rt.Multi([0, 0], rt.RT_MULTI_RCCL)


def test_comm_gather_single_rank(rt, orc, torch_cuda):
    """rt_comm with one rank: the RCCL send/recv to itself plus the scatter
    reproduce the compact band image as the full frame."""
    torch = torch_cuda
    s = rt.scene_prefix(rt.scene_builtin(1), 64)
    W, H, S, B = 120, 90, 3, 8
    cam = rt.camera_setup(s, W, H)
    ref = single(rt, torch, s, cam, W, H, S, B)
    comm = rt.Comm(0, rt.comm_unique_id(), 1, 0)
    try:
        full = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        fullp = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        comm.gather_bands(ref[1].data_ptr(), full.data_ptr(), W, H, 4, 8, stream=st)
        comm.gather_bands(ref[0].data_ptr(), fullp.data_ptr(), W, H, 16, 8, stream=st)
        torch.cuda.synchronize()
        assert torch.equal(full, ref[1]) and torch_equal_bits(fullp, ref[0])
    finally:
        comm.close()


def test_on_render_over_several_devices(rt, orc, torch_cuda):
    """OnRender (one-frame lag, reset on scene switch) driving rt_multi: the
    completed frames equal the oracle's progressive frames."""
    rt.on_init(devices=[0, 0, 0])
    try:
        W, H = 64, 56
        img = np.zeros((H, W), np.uint32)
        o = orc.scene_builtin(2)
        ocam = orc.camera(o, W, H)
        done, _, _ = rt.on_render(img, 2)
        assert not done
        for k in range(3):
            rt.on_render_wait()
            done, rays, _ = rt.on_render(img, 2)
            assert done
            _, ocur, orays = orc.render(o, ocam, W, H, frames=k + 1, max_bounce=5)
            assert np.array_equal(img.reshape(-1), ocur), k
        rt.on_render_wait()
    finally:
        rt.on_shutdown()


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_multi_back_to_back_continuations_gather_the_mean(rt, torch_cuda, devices):
    """Continuations enqueued with no host synchronisation (PreviousRayCount 0,
    S, 2S, 3S) that also gather the resident means: call k+1's traces overwrite
    the means call k's gather reads, so they must wait for it (the
    prev_gathered ordering on the copy / RCCL send events).  Each call's
    gathered mean and frame equal one device's render of (k + 1) S frames.
    [0] runs the RCCL transport (send/recv to itself), [0, 0, 0] peer copies."""
    torch = torch_cuda
    s = rt.scene_prefix(rt.scene_builtin(1), 64)
    W, H, S, B = 160, 96, 2, 8
    cam = rt.camera_setup(s, W, H)
    refs = [single(rt, torch, s, cam, W, H, (k + 1) * S, B) for k in range(4)]
    m = rt.Multi(devices)
    try:
        m.upload_scene(s)
        st = torch.cuda.current_stream().cuda_stream
        outs = []
        for k in range(4):
            cur = torch.zeros(W * H, dtype=torch.int32, device="cuda")
            prev = torch.full((W * H, 4), float("nan"), dtype=torch.float32, device="cuda")
            rays = torch.zeros(1, dtype=torch.int64, device="cuda")
            m.trace(cam, width=W, height=H, cur_ptr=cur.data_ptr(), prev_ptr=prev.data_ptr(),
                    rays_ptr=rays.data_ptr(), prev_count=k * S, frames=S, max_bounce=B, band_rows=8, stream=st)
            outs.append((prev, cur, rays))
        torch.cuda.synchronize()
    finally:
        m.close()
    total = 0
    for k, ((prev, cur, rays), ref) in enumerate(zip(outs, refs)):
        total += int(rays.item())
        assert total == ref[2], k
        assert torch_equal_bits(prev, ref[0]), ("running mean differs", k)
        assert torch_equal_bits(cur, ref[1]), ("RGBA8 differs", k)


def test_multi_accum_zero_restart_at_a_nonzero_count_continues_from_there(rt, torch_cuda):
    """RT_FLAG_ACCUM_ZERO with PreviousRayCount N > 0 folds its F frames with
    the weights of N, N + 1, ... (like rt_trace), so the continuation names
    N + F: N = 5, F = 2, then 3 more frames from 7; equal to one
    device doing the same two launches."""
    torch = torch_cuda
    s = rt.scene_prefix(rt.scene_builtin(1), 16)
    W, H, B = 64, 48, 4
    cam = rt.camera_setup(s, W, H)
    dev = rt.Device(0)
    try:
        dev.upload_scene(s)
        prev = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        cur = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        rays = torch.zeros(1, dtype=torch.int64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        for pc, f, az in ((5, 2, True), (7, 3, False)):
            dev.trace(cam, width=W, height=H, prev_ptr=prev.data_ptr(), cur_ptr=cur.data_ptr(),
                      rays_ptr=rays.data_ptr(), prev_count=pc, frames=f, max_bounce=B, band_rows=8,
                      accum_zero=az, stream=st)
        torch.cuda.synchronize()
    finally:
        dev.close()
    m = rt.Multi([0, 0])
    try:
        m.upload_scene(s)
        multi_render(rt, torch, m, cam, W, H, 2, B, prev_count=5, accum_zero=True)
        with pytest.raises(rt.RtError, match="holds 7 frames"):
            multi_render(rt, torch, m, cam, W, H, 3, B, prev_count=2)
        got = multi_render(rt, torch, m, cam, W, H, 3, B, prev_count=7)
    finally:
        m.close()
    assert torch_equal_bits(got[0], prev) and torch_equal_bits(got[1], cur)


def test_multi_reserve_means_no_allocation_in_later_calls(rt, orc, torch_cuda):
    """rt_multi_reserve sizes every device's images, launch buffers and the
    gather staging for a geometry: later calls of it (new cameras, P chosen per
    launch by the frame count) grow nothing (BufferGrowths constant on every
    device), report a gather time, and the slowest device's real launch info."""
    torch = torch_cuda
    s = rt.scene_prefix(rt.scene_builtin(1), 64)
    W, H, B = 200, 150, 8
    m = rt.Multi([0, 0, 0])
    try:
        m.upload_scene(s)
        m.reserve(W, H, 8, mean=True)
        st = torch.cuda.current_stream().cuda_stream
        cur = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        prev = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        rays = torch.zeros(1, dtype=torch.int64, device="cuda")
        m.trace(rt.camera_setup(s, W, H), width=W, height=H, cur_ptr=cur.data_ptr(), rays_ptr=rays.data_ptr(),
                frames=1, max_bounce=B, band_rows=8, accum_zero=True, stream=st)
        torch.cuda.synchronize()
        before = [m.shard_info(i)["BufferGrowths"] for i in range(3)]
        for frames, dist in ((1, 5.0), (4, None), (32, 2.5), (3, None)):
            cam = rt.camera_setup(s, W, H, distance=dist)
            m.trace(cam, width=W, height=H, cur_ptr=cur.data_ptr(), prev_ptr=prev.data_ptr(),
                    rays_ptr=rays.data_ptr(), frames=frames, max_bounce=B, band_rows=8, accum_zero=True, stream=st)
        torch.cuda.synchronize()
        after = [m.shard_info(i) for i in range(3)]
        assert [a["BufferGrowths"] for a in after] == before
        assert all(a["LanesPerPixel"] >= 1 for a in after)
        assert m.last_gather_ms() >= 0.0
    finally:
        m.close()


def test_multi_reserve_that_grows_the_mean_refuses_a_continuation(rt, orc, torch_cuda):
    """rt_multi_reserve growing the devices' resident running means discards
    them: after trace (geometry G) + reserve (larger) a continuation at G is
    RT_EINVAL instead of blending onto uninitialised memory, and a restart then
    continues bit-exactly (the oracle's frame)."""
    torch = torch_cuda
    s = rt.scene_prefix(rt.scene_builtin(1), 16)
    W, H, B = 64, 48, 6
    cam = rt.camera_setup(s, W, H)
    m = rt.Multi([0, 0])
    try:
        m.upload_scene(s)
        multi_render(rt, torch, m, cam, W, H, 2, B, prev_count=0, accum_zero=True)
        m.reserve(4 * W, 4 * H, 8)
        with pytest.raises(rt.RtError, match="no resident running mean"):
            multi_render(rt, torch, m, cam, W, H, 1, B, prev_count=2)
        multi_render(rt, torch, m, cam, W, H, 2, B, prev_count=0, accum_zero=True)
        got = multi_render(rt, torch, m, cam, W, H, 1, B, prev_count=2)
    finally:
        m.close()
    o = orc.scene_builtin(1).prefix(16)
    oprev, ocur, _ = orc.render(o, orc.camera(o, W, H), W, H, frames=3, max_bounce=B)
    assert np.array_equal(got[0].cpu().numpy().view(np.uint32).reshape(-1, 4), oprev.view(np.uint32))
    assert np.array_equal(got[1].cpu().numpy().view(np.uint32), ocur)


def test_on_render_multi_reserve_after_the_first_frame_restarts(rt, orc, torch_cuda):
    """with several devices, a reservation that grows the shards
    right after frame 0 (PreviousRayCount still 0) drops the resident means;
    the next OnRender call must restart the mean instead of continuing it
    (which rt_multi_trace refuses).  The frames handed out are the oracle's:
    the completed frame 0, the restarted frame 0, then frames 1 and 2."""
    rt.on_init(devices=[0, 0])
    try:
        W, H = 64, 48
        img = np.zeros((H, W), np.uint32)
        o = orc.scene_builtin(1)
        ocam = orc.camera(o, W, H)
        done, _, _ = rt.on_render(img, 1)
        assert not done
        rt.on_render_wait()
        rt.on_render_reserve(1920, 1088)  # past OnInit's 1280x720: the shards' means grow (and are dropped)
        got = []
        for _ in range(4):
            done, _, _ = rt.on_render(img, 1)
            assert done
            got.append(img.copy())
            rt.on_render_wait()
    finally:
        rt.on_shutdown()
    for k, frames in enumerate((1, 1, 2, 3)):
        _, ocur, _ = orc.render(o, ocam, W, H, frames=frames, max_bounce=5)
        assert np.array_equal(got[k].reshape(-1), ocur), k


def test_rccl_branch_over_eight_shards_of_one_gpu(loopback_rccl_result, rt):
    """rt_multi's RCCL transport (grouped ncclSend/ncclRecv of every shard's
    band image, running mean and ray count to devices[0], transfer streams, the
    two band-image slots and their sent events; main.cpp:851-856 /
    wasm/wasm.cpp:651-678's gather) over eight shards of this GPU, through the
    test-only loopback librccl.so.1 (tests/loopback_rccl: RCCL's point-to-point
    semantics as stream-ordered copies; the real RCCL refuses a device listed
    twice).  tests/loopback_rccl/multi_rccl_check, started by conftest before
    this process touched the GPU, traces BASELINE C2 (1920x1080, 256 spp, 64
    spheres, 8 bounces) with the gathered mean, an 8-frame continuation on the
    resident means and three restarts back to back, each compared byte for byte
    with one device's whole-frame render; C2's hashes and ray count must be the
    golden's (rendered by the reference itself).  rt_comm with several
    processes stays untested on a one-GPU box."""
    import json
    import pathlib
    rc, out = loopback_rccl_result
    assert out is not None and rc == 0, (rc, out)
    assert out["transport"] == "rccl" and out["devices"] == 8
    gold = json.loads((pathlib.Path(__file__).parent / "golden" / "oracle_regression.json").read_text())
    g = gold["c2_full_1920x1080x256"]
    a = out["a"]
    assert a["equal_one_device"] and a["rays"] == g["rays"] == 719275410
    assert a["fnv1a64_rgba8"] == g["fnv1a64_rgba8"] and a["fnv1a64_v4"] == g["fnv1a64_v4"]
    assert out["b"]["equal_one_device"] and out["b"]["resident_frames"] == 264
    assert out["c"]["equal_one_device"] == [True, True, True] and out["c"]["resident_frames"] == 3004
