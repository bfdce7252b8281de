"""Command-line applications of blendtorch.btt (``blendtorch-launch``: see
``launch.py``)."""
