"""AnimationController callback order (reference: tests/test_animation.py).

The reference's test body swallows every exception (tests/test_animation.py
:39-43) so it can never fail; here the sequence is asserted, for both the
blocking (--background) and the timer-driven UI loop (POST_PIXEL handler,
drawn twice per frame to exercise the duplicate-draw guard)."""
import pytest

from blendtorch import btt
from helpers import BLENDDIR, HEADLESS_BLENDER

EXPECTED = [
    'pre_play', 1,
    'pre_animation', 1, 'pre_frame', 1, 'post_frame', 1, 'pre_frame', 2, 'post_frame', 2,
    'pre_frame', 3, 'post_frame', 3, 'post_animation', 3,
    'pre_animation', 1, 'pre_frame', 1, 'post_frame', 1, 'pre_frame', 2, 'post_frame', 2,
    'pre_frame', 3, 'post_frame', 3, 'post_animation', 3,
    'post_play', 3,
]


def _capture(background, port):
    args = dict(scene='', script=BLENDDIR / 'anim.blend.py', named_sockets=['DATA'], background=background,
                start_port=port, blend_path=HEADLESS_BLENDER)
    with btt.BlenderLauncher(**args) as bl:
        ds = btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'], max_items=1, timeoutms=20000)
        return next(iter(ds))['seq']


@pytest.mark.background
def test_anim_callback_sequence(free_port):
    assert _capture(True, free_port) == EXPECTED


def test_anim_callback_sequence_ui(free_port):
    assert _capture(False, free_port) == EXPECTED
