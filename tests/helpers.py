"""Shared test helpers: the headless Blender stand-in and its scene files."""
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
BLENDDIR = Path(__file__).resolve().parent / 'blender'
# directory holding the headless `blender` executable (blendtorch.btb.headless)
HEADLESS_BLENDER = str(ROOT / 'pytorch-blender_amd' / 'blendtorch' / 'btb' / 'headless' / 'bin')
