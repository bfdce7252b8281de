#!/bin/bash
# Install a Blender release for the real-Blender producer path (the bundled
# headless emulation and C++ stand-ins need none of this).  Mirrors the
# reference's scripts/install_blender.sh: cache the tarball under
# ~/.blender-cache, unpack into $HOME, write `.envs` with the PATH export.
#
#   scripts/install_blender.sh [VERSION] [TARBALL]
#
# VERSION defaults to 2.90.0 (the reference's CI version).  With TARBALL the
# archive is taken from disk (offline hosts); otherwise it is downloaded.
set -euo pipefail
VERSION="${1:-2.90.0}"
MAJMIN="${VERSION%.*}"
NAME="blender-${VERSION}-linux64"
NAMETAR="${NAME}.tar.xz"
CACHE="${HOME}/.blender-cache"
TAR="${CACHE}/${NAMETAR}"
URL="https://download.blender.org/release/Blender${MAJMIN}/${NAMETAR}"

echo "Installing Blender ${NAME}"
mkdir -p "$CACHE"
if [ $# -ge 2 ]; then
    cp "$2" "$TAR"
elif [ ! -f "$TAR" ]; then
    if command -v wget >/dev/null; then wget -O "$TAR" "$URL"; else curl -L -o "$TAR" "$URL"; fi
fi
tar -xf "$TAR" -C "$HOME"
echo "export PATH=\"\${PATH}:${HOME}/${NAME}\"" > .envs
echo "wrote .envs; next: source .envs && blender --background --python scripts/install_btb.py"
