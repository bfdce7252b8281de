"""Blender-side units under the headless emulation: arguments, Signal,
OffScreenRenderer (gamma/flip vs the GPU decode LUT), AnimationController
details (rewind, physics range, manual loop)."""
import numpy as np
import pytest

from blendtorch import btb, ops
from blendtorch.btb import headless


def test_parse_blendtorch_args():
    argv = ['blender', '--python', 'x.py', '--', '-btid', '2', '-btseed', '7', '-btsockets', 'DATA=tcp://a:1',
            'GYM=tcp://b:2', '--x', '3']
    args, rem = btb.parse_blendtorch_args(argv)
    assert args.btid == 2 and args.btseed == 7
    assert args.btsockets == {'DATA': 'tcp://a:1', 'GYM': 'tcp://b:2'}
    assert rem == ['--x', '3']
    with pytest.raises(ValueError):
        btb.parse_blendtorch_args(['blender', '-btid', '1'])


def test_signal_add_remove_invoke():
    got = []
    s = btb.Signal()
    h = s.add(lambda a, b: got.append(a * b), b=3)
    s.add(lambda a: got.append(-a))
    s.invoke(4)
    assert got == [12, -4]
    s.remove(h)
    s.invoke(1)
    assert got == [12, -4, -1]


def test_offscreen_render_modes_and_gamma():
    headless.install('cube.blend')
    cam = btb.Camera()
    assert cam.shape == (480, 640)
    off = btb.OffScreenRenderer(camera=cam, mode='rgba', origin='lower-left')
    raw = off.render().copy()
    assert raw.shape == (480, 640, 4) and (raw[..., 3] == 255).all()
    ul = btb.OffScreenRenderer(camera=cam, mode='rgb').render()
    assert np.array_equal(ul, raw[::-1, :, :3])
    g = btb.OffScreenRenderer(camera=cam, mode='rgba', gamma_coeff=2.2).render()
    lut = ops.gamma_lut(2.2)
    assert np.array_equal(g[..., :3], lut[raw[::-1, :, :3]])     # bit-exact with the GPU LUT
    assert np.array_equal(g[..., 3], raw[::-1, :, 3])            # alpha untouched
    # the cube is visible near the image centre
    assert ul[200:280, 280:360].std() > 5


def test_animation_rewind_and_physics_range():
    bpy = headless.install('falling_cubes.blend')
    anim = btb.AnimationController()
    frames = []
    anim.pre_frame.add(lambda: frames.append(anim.frameid))
    state = {'rewound': False}

    def post():
        if anim.frameid == 3 and not state['rewound']:
            state['rewound'] = True
            anim.rewind()
    anim.post_frame.add(post)
    anim.play(frame_range=(1, 4), num_episodes=1, use_animation=False)
    assert bpy.context.scene.rigidbody_world.point_cache.frame_end == 4
    assert frames[:3] == [1, 2, 3] and frames[3] == 1 and frames[-1] == 4


def test_utils_coordinates():
    bpy = headless.install('cube.blend')
    cube = bpy.data.objects['Cube']
    cube.location = (1, 2, 3)
    w = btb.utils.world_coordinates(cube)
    assert np.allclose(w - btb.utils.object_coordinates(cube), [1, 2, 3])
    bb = btb.utils.bbox_world_coordinates(cube)
    assert bb.shape == (8, 3) and np.allclose(bb.min(0), [0, 1, 2])
    x = np.random.rand(5, 3)
    assert np.allclose(btb.utils.dehom(btb.utils.hom(x, 2.0)), x / 2.0)
    p = btb.utils.random_spherical_loc(radius_range=(2, 2))
    assert abs(np.linalg.norm(p) - 2) < 1e-9
    cam = btb.Camera()
    vis = btb.utils.compute_object_visibility(cube, cam, N=10)
    assert 0.0 <= vis <= 1.0


def test_value_table_arithmetic_forms_reproduce_reference_tables():
    """ops.build_table: every common decode config gets the kernels'
    arithmetic path (mode 1), and the verified per-channel form -- applied to
    the lane-private gamma table exactly as the kernels index it -- equals
    the fp32 reference table bit for bit (so the LDS-free / conflict-free
    decode stays bit-exact)."""
    import numpy as np
    from blendtorch import ops
    cfgs = [ops.DecodeConfig.unit(channels='rgb', gamma=2.2),
            ops.DecodeConfig.unit(channels='rgba', gamma=2.2, dtype='bfloat16', layout='nhwc'),
            ops.DecodeConfig.densityopt(channels='rgb'),
            ops.DecodeConfig.densityopt(channels=(0, 1, 2, 2), dtype='bfloat16', layout='nhwc'),
            ops.DecodeConfig.densityopt(channels='rgb', gamma=2.2),
            ops.DecodeConfig.raw(), ops.DecodeConfig.raw(channels='rgb'),
            ops.DecodeConfig(channels='bgr', mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225), scale=1 / 255),
            ops.DecodeConfig(channels='rgba', gamma=1.8, color_matrix=np.eye(4).tolist()),
            ops.DecodeConfig.unit(channels='rgb', gamma=2.2, color_jitter=ops.ColorJitter(0.4, 0.4, 0.4, 0.1))]
    import os
    os.environ['BLENDTORCH_DECODE_XFORM'] = '1'      # the forced arithmetic path (auto keeps the table for gamma)
    try:
        tables = [ops.build_table(cfg) for cfg in cfgs]
    finally:
        del os.environ['BLENDTORCH_DECODE_XFORM']
    assert ops.build_table(ops.DecodeConfig.unit(channels='rgb'))[ops.XF_HEADER] == 1.0          # auto: no LDS
    assert ops.build_table(ops.DecodeConfig.unit(channels='rgb', gamma=2.2))[ops.XF_HEADER] == 0.0
    for cfg, t in zip(cfgs, tables):
        assert t.shape == (ops.TABLE_FLOATS,) and t.dtype == np.float32
        assert t[ops.XF_HEADER] == 1.0, cfg
        lut = ops.build_lut(cfg)
        hdr = t[ops.XF_HEADER:ops.XF_HEADER + 26]
        gw = t[ops.XF_GAMMA:ops.XF_GAMMA + 64].view(np.uint32)
        tab = np.repeat(gw, 32).view(np.uint8)                  # word i = gamma dword i >> 5 (32 copies)
        assert hdr[1] in (0.0, 32.0)
        nch = 4 if cfg.colour_kernel else cfg.cout
        v = np.arange(256)
        from blendtorch import _native
        for lane in (0, 7, 31):
            for c in range(nch):
                if hdr[2 + c]:
                    x = tab[(v >> 2) * 128 + lane * 4 + (v & 3)].astype(np.float32)
                else:
                    x = v.astype(np.float32)
                op, a, b, d, r = int(hdr[6 + c]), hdr[10 + c], hdr[14 + c], hdr[18 + c], hdr[22 + c]
                z = np.array([_native.xform_apply(op, a, b, d, r, float(xi)) for xi in x], dtype=np.float32)
                assert op in (0, 1, 3) or cfg.std is not None, (cfg, op)     # division only as the last resort
                assert np.array_equal(z.view(np.uint32), lut[c].view(np.uint32)), (cfg, c, lane)


def test_color_jitter_matrix_and_configs():
    """ops.color_jitter_matrix: identity factors give the identity, every
    transform keeps grey grey (rows sum to b*c, bias (1-c)*pivot), and hue /
    saturation compose as documented; DecodeConfig validates the per-image
    transforms; the jitter reference with identity factors is the plain decode."""
    import numpy as np
    import pytest
    import torch
    from blendtorch import ops
    M, b = ops.color_jitter_matrix([1, 1, 1, 0])
    np.testing.assert_allclose(M, np.eye(4), atol=1e-7)
    assert not b.any()
    rng = np.random.default_rng(0)
    for _ in range(20):
        f = [rng.uniform(0.5, 1.5), rng.uniform(0.5, 1.5), rng.uniform(0, 2), rng.uniform(-0.5, 0.5)]
        M, b = ops.color_jitter_matrix(f, 0.5)
        np.testing.assert_allclose(M[:3, :3].sum(1), f[0] * f[1], rtol=1e-5)
        np.testing.assert_allclose(b[:3], (1 - f[1]) * 0.5, rtol=1e-6)
        assert M[3].tolist() == [0, 0, 0, 1] and not M[:3, 3].any()
    # saturation 0: every output channel is the luminance
    M, _ = ops.color_jitter_matrix([1, 1, 0, 0.3])
    np.testing.assert_allclose(M[:3, :3], np.tile([0.213, 0.715, 0.072], (3, 1)), atol=1e-6)
    # a full turn of hue is the identity
    M, _ = ops.color_jitter_matrix([1, 1, 1, 0.5])
    M2, _ = ops.color_jitter_matrix([1, 1, 1, -0.5])
    np.testing.assert_allclose(M, M2, atol=1e-6)
    f = ops.jitter_factors(3, [0.4, 0.2, 0.0, 0.1], 50)
    assert f.shape == (50, 4) and (f[:, 0] >= 0.6).all() and (f[:, 0] <= 1.4).all()
    assert (f[:, 2] == 1).all() and (np.abs(f[:, 3]) <= 0.1).all()
    np.testing.assert_array_equal(f, ops.jitter_factors(3, [0.4, 0.2, 0.0, 0.1], 50))
    assert not np.array_equal(f, ops.jitter_factors(4, [0.4, 0.2, 0.0, 0.1], 50))
    with pytest.raises(ValueError):
        ops.DecodeConfig.unit(channels='bgr', color_jitter=ops.ColorJitter(0.1))
    with pytest.raises(ValueError):
        ops.DecodeConfig(color_jitter=ops.ColorJitter(0.1), color_matrix=np.eye(4))
    with pytest.raises(ValueError):
        ops.ColorJitter(hue=0.7)
    with pytest.raises(ValueError):
        ops.DecodeConfig(channels='rgba', color_matrices=np.zeros((2, 3, 4)))
    cfg = ops.DecodeConfig(channels='rgba', color_matrices=np.stack([np.eye(4)] * 3))
    assert cfg.cout == 4 and cfg.colour_kernel and len(cfg.color_biases) == 3
    x = torch.randint(0, 256, (2, 8, 16, 4), dtype=torch.uint8)
    jc = ops.DecodeConfig.unit(channels='rgb', gamma=2.2, color_jitter=ops.ColorJitter(0.3, 0.3, 0.3, 0.1))
    assert jc.cout == 3 and jc.jitter_pivot == 0.5
    got = ops.reference_decode(x, jc, jitter=[[1, 1, 1, 0]] * 2)
    want = ops.reference_decode(x, ops.DecodeConfig.unit(channels='rgb', gamma=2.2))
    torch.testing.assert_close(got, want, rtol=1e-6, atol=1e-6)
