"""Per-phase breakdown of the f32 render kernel from the RRT_PHASE_TIMING debug builds
(tools/phase_breakdown.sh: gpurun_out/phase/<config>_pt<k>.json, one 64-spp launch each).

Counter slots 2..4 of each debug build (rrt_kernel.hip header):
  pt1 wave cycles in refill + segment start / traversal (node steps + leaf batches) / shading + next ray
  pt2 node-step wave-iterations x64 / lanes stepping / outer iterations (per wave)
  pt3 leaf-loop wave-iterations x64 / lanes testing / lanes reaching the root code (disc >= 0)
  pt4 shading passes x64 / shading lanes / rejection-loop (random_unit_vector) wave-iterations x64
  pt5 dielectric-branch entries x64 / dielectric lanes / metal-branch entries x64
  pt6 metal lanes / sky-branch entries x64 / sky lanes
  pt7 camera-ray entries after a path end x64 / their lanes / defocus-disk wave-iterations x64
  pt8 node-step wave-iterations x64 / those whose stepping lanes all visit one node x64 / their lanes

VALU wave-instructions per iteration are static counts from the shipped kernel's ISA (the C2 class
rrt_render<LDS, 16-bit stack, BVH2, 6 waves, book-1 untextured, 512>; `make -C rustraytrace_amd/csrc
asm`): a node step 45, a leaf iteration 17 + 29 in the root code, a rejection-loop iteration 35, a
disk iteration 23. VALU share = iterations x instructions / the launch's measured VALU count
(SQ_INSTS_VALU per ray from profiles/issue_<config>.json x rays): an estimate, the rest of the
stream (refill, shading outside the loop, the camera ray) is the remainder.

    python tools/phase_breakdown.py gpurun_out/phase <config> <out_json>
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VALU = {"node": 45, "leaf": 17, "root": 29, "reject": 35, "disk": 23}


def main(d, config, out):
    c = {k: json.load(open(os.path.join(d, f"{config}_pt{k}.json")))["counters"] for k in range(1, 9)}
    rays = json.load(open(os.path.join(d, f"{config}_pt1.json")))["rays_per_launch"]
    s = lambda k, slot: c[k][("node_visits", "box_tests", "sphere_tests")[slot]]
    cyc = [s(1, 0), s(1, 1), s(1, 2)]
    node_it, node_lanes = s(2, 0) / 64, s(2, 1)
    leaf_it, leaf_lanes, root_lanes = s(3, 0) / 64, s(3, 1), s(3, 2)
    shade_it, shade_lanes, rej_it = s(4, 0) / 64, s(4, 1), s(4, 2) / 64
    diel_it, diel_lanes, metal_it = s(5, 0) / 64, s(5, 1), s(5, 2) / 64
    metal_lanes, sky_it, sky_lanes = s(6, 0), s(6, 1) / 64, s(6, 2)
    cam_it, cam_lanes, disk_it = s(7, 0) / 64, s(7, 1), s(7, 2) / 64
    uni_it, uni_lanes = s(8, 1) / 64, s(8, 2)
    scatter_lanes = shade_lanes - sky_lanes - diel_lanes  # Lambertian + metal (+ emitters: none in C2/C5)
    issue = json.load(open(os.path.join(ROOT, "profiles", f"issue_{config}.json")))
    valu_total = issue["valu_insts_per_ray"] * rays
    est = {
        "node_steps": node_it * VALU["node"],
        "leaf_iterations": leaf_it * VALU["leaf"] + leaf_it * VALU["root"] * min(1.0, root_lanes / leaf_it),
        "rejection_loop": rej_it * VALU["reject"],
        "defocus_disk_loop": disk_it * VALU["disk"],
    }
    rec = {
        "config": config, "spp": 64, "rays_per_launch": rays,
        "wave_cycle_share": {"refill_and_segment_start": cyc[0] / sum(cyc), "traversal": cyc[1] / sum(cyc),
                             "shading_and_next_ray": cyc[2] / sum(cyc)},
        "phases": {
            "node_step": {"wave_iterations": node_it, "lanes_per_iteration": node_lanes / node_it,
                          "per_ray": node_it / rays,
                          "single_node_steps_frac": uni_it / node_it,
                          "lanes_per_single_node_step": uni_lanes / max(uni_it, 1)},
            "leaf_iteration": {"wave_iterations": leaf_it, "lanes_per_iteration": leaf_lanes / leaf_it,
                               "root_code_lanes_per_iteration": root_lanes / leaf_it,
                               "tests_per_ray": leaf_lanes / rays},
            "shading_pass": {"passes": shade_it, "lanes_per_pass": shade_lanes / shade_it,
                             "sky_lanes_per_pass": sky_lanes / shade_it, "sky_entries_frac": sky_it / shade_it,
                             "dielectric_lanes_per_entry": diel_lanes / max(diel_it, 1),
                             "dielectric_entries_frac": diel_it / shade_it,
                             "metal_lanes_per_entry": metal_lanes / max(metal_it, 1),
                             "metal_entries_frac": metal_it / shade_it,
                             "scatter_lanes_per_pass": scatter_lanes / shade_it},
            "rejection_loop": {"wave_iterations": rej_it, "iterations_per_pass": rej_it / shade_it,
                               "lanes_per_iteration_expected": scatter_lanes * (6.0 / 3.14159265) / rej_it,
                               "note": "lane-candidates = scatter lanes x 6/pi (the acceptance of a point of "
                                       "[-1,1)^3 in the unit ball is pi/6)"},
            "camera_ray_after_path_end": {"entries": cam_it, "lanes_per_entry": cam_lanes / max(cam_it, 1),
                                          "disk_iterations": disk_it, "disk_iterations_per_entry": disk_it / max(cam_it, 1),
                                          "disk_lanes_per_iteration_expected": cam_lanes * (4.0 / 3.14159265) / max(disk_it, 1)},
        },
        "valu_estimate": {k: {"wave_instructions": v, "share_of_launch": v / valu_total} for k, v in est.items()},
        "valu_per_iteration_static": VALU,
        "valu_total_from_issue_record": valu_total,
        "source": "tools/phase_breakdown.sh (RRT_PHASE_TIMING 1..8 debug builds, one 64-spp launch each)",
    }
    rec["valu_estimate"]["rest"] = {"wave_instructions": valu_total - sum(est.values()),
                                    "share_of_launch": 1 - sum(est.values()) / valu_total}
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
