"""Falling-cubes producer, run inside Blender (or the headless emulation).

Scene ``falling_cubes.blend`` holds a collection ``Cubes`` of rigid bodies.
Each one gets its own random colour once. At the start of every episode, all
of them are dropped again from random positions above the ground, and
physics lets them fall. Every frame is published with the projected corners
of all cubes (``xy``, 8 per cube) and the frame id. Same behaviour as the
reference scene script; the native stand-in is ``cubesim --scene falling_cubes``.
"""
import bpy
import numpy as np

from blendtorch import btb

EPISODE = (0, 100)
DROP_LOW, DROP_HIGH = (-3.0, -3.0, 6.0), (3.0, 3.0, 12.0)


def colour_cubes(cubes, rng):
    """One fresh material with a random opaque diffuse colour per cube."""
    for n, cube in enumerate(cubes):
        material = bpy.data.materials.new(name=f'random{n}')
        material.diffuse_color = (*rng.random(3), 1.0)
        cube.data.materials.append(material)
        cube.active_material = material


def drop(cubes, rng):
    """pre_animation: new start pose for every cube."""
    positions = rng.uniform(DROP_LOW, DROP_HIGH, size=(len(cubes), 3))
    angles = rng.uniform(-np.pi, np.pi, size=(len(cubes), 3))
    for cube, p, a in zip(cubes, positions, angles):
        cube.location = p
        cube.rotation_euler = a


def main():
    btargs, _ = btb.parse_blendtorch_args()
    np.random.seed(btargs.btseed)   # the reference seeds numpy's global state
    rng = np.random
    cubes = list(bpy.data.collections['Cubes'].objects)
    colour_cubes(cubes, rng)

    camera = btb.Camera()
    renderer = btb.OffScreenRenderer(camera=camera, mode='rgb')
    renderer.set_render_style(shading='RENDERED', overlays=False)
    publisher = btb.DataPublisher(btargs.btsockets['DATA'], btargs.btid)
    anim = btb.AnimationController()

    def publish_frame():
        publisher.publish(image=renderer.render(), xy=camera.object_to_pixel(*cubes), frameid=anim.frameid)

    anim.pre_animation.add(drop, cubes, rng)
    anim.post_frame.add(publish_frame)
    anim.play(frame_range=EPISODE, num_episodes=-1, use_animation=not bpy.app.background)


main()
