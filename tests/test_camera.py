"""Camera projection golden numbers (reference: tests/test_camera.py:9-49).

The reference scene tests/blender/cam.blend: 640x480, CamOrtho (ortho_scale
4) and CamProj (lens 50, sensor 36) at (0,0,7) looking down -Z, unit cube
at the origin, clip 1..10 (values recovered in SURVEY.md §4)."""
import numpy as np
import pytest
from numpy.testing import assert_allclose

from blendtorch import btt
from helpers import BLENDDIR, HEADLESS_BLENDER

ORTHO_XY = np.array([[480., 80], [480., 80], [480., 400], [480., 400], [160., 80], [160., 80], [160., 400],
                     [160., 400]])
PROJ_XY = np.array([[468.148, 91.851], [431.111, 128.888], [468.148, 388.148], [431.111, 351.111],
                    [171.851, 91.851], [208.888, 128.888], [171.851, 388.148], [208.888, 351.111]])
Z = np.array([6., 8, 6, 8, 6, 8, 6, 8])


@pytest.mark.background
def test_projection(free_port):
    args = dict(scene=BLENDDIR / 'cam.blend', script=BLENDDIR / 'cam.blend.py', num_instances=1,
                named_sockets=['DATA'], background=True, start_port=free_port, blend_path=HEADLESS_BLENDER)
    with btt.BlenderLauncher(**args) as bl:
        item = next(iter(btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'], max_items=2)))
    assert_allclose(item['ortho_xy'], ORTHO_XY, atol=1e-2)
    assert_allclose(item['ortho_z'], Z, atol=1e-2)
    assert_allclose(item['proj_xy'], PROJ_XY, atol=1e-2)
    assert_allclose(item['proj_z'], Z, atol=1e-2)
    assert_allclose(item['obj_px'], PROJ_XY, atol=1e-2)
    assert item['bbox_px'].shape == (8, 2)


def test_projection_in_process():
    """Same numbers in-process through the headless bpy emulation."""
    from blendtorch.btb import headless
    headless.install('cam.blend')
    import bpy
    from blendtorch.btb.camera import Camera
    from blendtorch.btb import utils
    cam = Camera(bpy.data.objects['CamProj'])
    xyz = utils.world_coordinates(bpy.data.objects['Cube'])
    ndc, z = cam.world_to_ndc(xyz, return_depth=True)
    assert_allclose(cam.ndc_to_pixel(ndc), PROJ_XY, atol=1e-2)
    assert_allclose(z, Z, atol=1e-6)
    ll = cam.ndc_to_pixel(ndc, origin='lower-left')
    assert_allclose(ll[:, 1], 480 - PROJ_XY[:, 1], atol=1e-2)
    # look_at keeps the camera pointed at the target
    cam.look_at(look_at=(0, 0, 0), look_from=(3, -3, 4))
    px = cam.ndc_to_pixel(cam.world_to_ndc(np.zeros((1, 3))))
    assert_allclose(px, [[320, 240]], atol=1e-6)


def test_camera_matches_gpu_project_reference():
    """btb.Camera math == blendtorch.ops.reference_project (used for the GPU kernel)."""
    from blendtorch.btb import headless
    headless.install('cube.blend')
    import bpy
    from blendtorch.btb.camera import Camera
    from blendtorch.btb import utils
    from blendtorch import ops
    cam = Camera()
    xyz = utils.world_coordinates(bpy.data.objects['Cube'])
    ndc, z = cam.world_to_ndc(xyz, return_depth=True)
    px = cam.ndc_to_pixel(ndc)
    PV = np.asarray(cam.proj_matrix @ cam.view_matrix)
    rpx, rz = ops.reference_project(xyz, PV, np.asarray(cam.view_matrix), 640, 480)
    assert_allclose(rpx.numpy(), px, atol=1e-6)
    assert_allclose(rz.numpy(), z, atol=1e-9)
