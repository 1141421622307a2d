"""Generate the committed fixtures under tests/golden/ from data files the reference holds.

Run in the build container only (it reads /root/reference, which the GPU box does not have):
    python tests/golden/make_fixtures.py
Outputs:
  earthmap_rgb8.npz       earthmap.jpg (src/Scenes.hs:159) decoded to RGB8 by Pillow/libjpeg. The
                          reference decodes with JuicyPixels; decoders differ by +-1-2 levels, so
                          texel parity with the reference is UNPINNED (hard parts).
  cornell1000_blocks.npz  10x10-block means (and stds) of cornellBox1000.png, the reference's own
                          render of makeCornellBoxScene at 500x500, 1000 spp, depth 50 (app/Main.hs).
                          A statistical fixture: 499 of its columns were clock-seeded.
"""
import os

import numpy as np
from PIL import Image

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    earth = np.asarray(Image.open(os.path.join(REF, "earthmap.jpg")).convert("RGB"), dtype=np.uint8)
    np.savez_compressed(os.path.join(OUT, "earthmap_rgb8.npz"), rgb=earth)
    im = np.asarray(Image.open(os.path.join(REF, "cornellBox1000.png")).convert("RGB"), dtype=np.float64)
    h, w, _ = im.shape
    b = im.reshape(h // 10, 10, w // 10, 10, 3)
    np.savez_compressed(os.path.join(OUT, "cornell1000_blocks.npz"), mean=b.mean(axis=(1, 3)),
                        std=b.std(axis=(1, 3)), image_mean=im.reshape(-1, 3).mean(0), shape=np.array(im.shape))
    print("earth", earth.shape, "cornell blocks", b.shape)


if __name__ == "__main__":
    main()
