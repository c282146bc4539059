"""Find the first (pixel, sample) where the GPU and the oracle's KBVH twin differ for a scene
built by a Python expression, e.g.
    python tools/debug_pixel.py "rrt.rest_of_your_life_scene(dict(image_width=64, samples_per_pixel=25, max_depth=50))"
Prints the pixel, the sample index and both single-sample results."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    import rustraytrace_amd as rrt
    from oracle import oracle
    from rustraytrace_amd.render import build_bvh
    from test_gpu_parity import gpu_tile

    for w in os.environ.get("WARMUP", "").split(";"):  # scenes rendered first in this process
        if w:
            rrt.render(eval(w, {"rrt": rrt, "np": np}))
    sc = eval(sys.argv[1], {"rrt": rrt, "np": np})
    nodes, order, info = build_bvh(sc)
    gpu = rrt.render(sc)
    ref, _, _ = oracle.render_kbvh(sc, nodes, order, info, threads=16)
    bad = np.argwhere(np.any(gpu.astype(np.float64) != ref, axis=-1))
    print("differing pixels:", len(bad), bad[:8].tolist())
    if not len(bad):
        return
    y, x = bad[0]
    for s in range(sc.spp):
        g, _, _, _ = gpu_tile(sc, s0=s, s1=s + 1)
        r, _, _ = oracle.render_kbvh(sc, nodes, order, info, rows=(int(y), int(y) + 1), samples=(s, s + 1))
        if not np.array_equal(g[y, x].astype(np.float64), r[0, x]):
            print(f"pixel x={x} y={y} sample {s}: gpu {g[y, x].tolist()} oracle {r[0, x].tolist()}")
            if len(sys.argv) > 2:
                with open(sys.argv[2], "w") as f:
                    f.write(f"{x} {y} {s}\n")
            return
    print("no single sample differs (accumulation order?)")


if __name__ == "__main__":
    main()
