// Keyframe-delta tile codec for same-host frames (shared-memory ring).
//
// A static camera renders the same background in every frame; only the
// pixels the moving objects cover change.  A producer that knows its
// background (the "key" frame) publishes it ONCE in a shared-memory segment of
// its own; every frame then goes into its ring slot as
//
//   [ u32 n | u32 pos[ntiles] | pad to 256 B | payload tile 0 | tile 1 ... ]
//
// over a grid of kTile x kTile pixel tiles of the stored (HWC u8) image
// (tile index t = ty * (W / kTile) + tx): payload tile k < n replaces tile
// pos[k] and is stored as kTile rows of kTile*C contiguous bytes; every other
// tile equals the key frame.  The encoding is lossless; it needs
// H % kTile == 0 and W % kTile == 0.
//
// Why: the GPU loader reads frames straight out of pinned host memory over
// PCIe, and that link is the pipeline's ceiling (~50 GB/s on MI355X, see
// profiles/direct_host_read.md).  The key frame sits in HBM after its first
// use, so only the changed tiles cross PCIe: the GPU fills each output image
// from the key frame decoded once in HBM, then a scatter kernel decodes the
// payload tiles into place -- a tile's position and its pixels are two
// independent loads (no dependent map lookup over PCIe), and each wave reads
// whole tiles (1 KiB contiguous for RGBA).
//
// The descriptor of an encoded frame (_btshm, csrc/transport/shmring.h) gets
// a 9th element ("tile16", key segment name, key generation).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>

namespace btn {
namespace tiledelta {

constexpr int kTile = 16;
constexpr const char* kName = "tile16";

inline bool supported(int H, int W, int C) { return H > 0 && W > 0 && H % kTile == 0 && W % kTile == 0 && C >= 1 && C <= 4; }
inline size_t ntiles(int H, int W) { return size_t(H / kTile) * size_t(W / kTile); }
// byte offset of payload tile 0 (count + position list rounded up to 256 B)
inline size_t payload_offset(int H, int W) { return ((ntiles(H, W) + 1) * 4 + 255) & ~size_t(255); }
inline size_t tile_bytes(int C) { return size_t(kTile) * kTile * C; }
// worst case: every tile in the payload
inline size_t max_bytes(int H, int W, int C) { return payload_offset(H, W) + ntiles(H, W) * tile_bytes(C); }

// Encode `frame` against `key` (both H*W*C, row-major HWC) into `out`
// (max_bytes capacity).  Only tiles that intersect the row/column range
// [y0, y1] x [x0, x1] (inclusive, stored-row coordinates) are compared; the
// caller guarantees every pixel outside it equals the key.  An empty range
// (y1 < y0) yields an all-key frame.  Returns the bytes written.
inline size_t encode(const uint8_t* frame, const uint8_t* key, int H, int W, int C, int y0, int y1, int x0, int x1,
                     uint8_t* out) {
  const int tx_n = W / kTile, ty_n = H / kTile;
  uint32_t* pos = reinterpret_cast<uint32_t*>(out) + 1;
  uint8_t* pay = out + payload_offset(H, W);
  const size_t row = size_t(kTile) * C;
  uint32_t k = 0;
  if (y1 >= y0 && x1 >= x0) {
    y0 = y0 < 0 ? 0 : y0, x0 = x0 < 0 ? 0 : x0;
    y1 = y1 >= H ? H - 1 : y1, x1 = x1 >= W ? W - 1 : x1;
    for (int ty = y0 / kTile; ty <= y1 / kTile && ty < ty_n; ++ty)
      for (int tx = x0 / kTile; tx <= x1 / kTile && tx < tx_n; ++tx) {
        const size_t base = (size_t(ty) * kTile * W + size_t(tx) * kTile) * C;
        bool same = true;
        for (int r = 0; r < kTile && same; ++r)
          same = std::memcmp(frame + base + size_t(r) * W * C, key + base + size_t(r) * W * C, row) == 0;
        if (same) continue;
        uint8_t* dst = pay + size_t(k) * tile_bytes(C);
        for (int r = 0; r < kTile; ++r) std::memcpy(dst + size_t(r) * row, frame + base + size_t(r) * W * C, row);
        pos[k++] = uint32_t(ty * tx_n + tx);
      }
  }
  reinterpret_cast<uint32_t*>(out)[0] = k;
  return payload_offset(H, W) + size_t(k) * tile_bytes(C);
}

// Payload tile count of a well-formed encoded frame, or -1 when the count or
// a position is out of range for an H x W frame whose slot holds `cap` bytes.
inline long check(const uint8_t* enc, int H, int W, int C, size_t cap) {
  const uint32_t* hdr = reinterpret_cast<const uint32_t*>(enc);
  const size_t nt = ntiles(H, W);
  if (cap < payload_offset(H, W) || hdr[0] > nt || payload_offset(H, W) + size_t(hdr[0]) * tile_bytes(C) > cap)
    return -1;
  for (uint32_t k = 0; k < hdr[0]; ++k)
    if (hdr[1 + k] >= nt) return -1;
  return long(hdr[0]);
}

// Expand an encoded frame into `out` (H*W*C).
inline void expand(const uint8_t* enc, const uint8_t* key, int H, int W, int C, uint8_t* out) {
  const int tx_n = W / kTile;
  const uint32_t* hdr = reinterpret_cast<const uint32_t*>(enc);
  const uint8_t* pay = enc + payload_offset(H, W);
  const size_t row = size_t(kTile) * C;
  std::memcpy(out, key, size_t(H) * W * C);
  for (uint32_t k = 0; k < hdr[0]; ++k) {
    const int ty = int(hdr[1 + k]) / tx_n, tx = int(hdr[1 + k]) % tx_n;
    const uint8_t* src = pay + size_t(k) * tile_bytes(C);
    const size_t base = (size_t(ty) * kTile * W + size_t(tx) * kTile) * C;
    for (int r = 0; r < kTile; ++r) std::memcpy(out + base + size_t(r) * W * C, src + size_t(r) * row, row);
  }
}

}  // namespace tiledelta
}  // namespace btn
