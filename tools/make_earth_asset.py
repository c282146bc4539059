"""Decode the reference's images/earthmap.jpg (rtw_image.rs:57-67 `image::open(..).to_rgb8()`)
once, here, into the RGB8 asset the HIP backend and the oracle both read, so they see
identical bytes. The reference decodes with zune-jpeg 0.5.12 (Cargo.lock:1390); PIL uses
libjpeg-turbo, so texel parity with the reference's own decode is unpinned.

    python tools/make_earth_asset.py /root/reference/images/earthmap.jpg
"""
import hashlib
import sys

import numpy as np
from PIL import Image

EXPECTED_SHA256 = "a8cdc92a168d554ddc693785d31f5e251063724f44099571d7fbce3b43d44c45"


def main(src: str, dst: str = "rustraytrace_amd/assets/earthmap_rgb8.npz") -> None:
    rgb = np.asarray(Image.open(src).convert("RGB"), dtype=np.uint8)
    digest = hashlib.sha256(rgb.tobytes()).hexdigest()
    assert digest == EXPECTED_SHA256, digest
    np.savez_compressed(dst, rgb8=rgb)
    print(dst, rgb.shape, digest)


if __name__ == "__main__":
    main(*sys.argv[1:])
