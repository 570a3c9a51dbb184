#!/usr/bin/env python3
"""Generates tests/golden/placements.json: the oracle's outputs on
BASELINE.json configs 1-5 (assign[] in full for configs 1, 2, 3, 5; sha256 of
assign / cap / occ for all). These pin the oracle (and through it the GPU
engine) against regressions; they are outputs of this build's rules, not of
the reference (see DESIGN.md §6 for what the reference pins).

Run:  python tests/golden/make_placement_fixtures.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from jobset_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    out = {}
    for cfg, fn in synth.CONFIGS.items():
        p = fn()
        a, cap, occ = O.place_c(p)
        rec = {"name": p.name, "nodes": p.nodes.n_nodes, "leaves": p.topology.n_leaves, "jobs": p.n_jobs,
               "placed": int((a >= 0).sum()), "assign_sha256": digest(a.astype(np.int32)),
               "cap_sha256": digest(cap.astype(np.uint32)), "occ_sha256": digest(occ.astype(np.uint32)),
               "snapshot_sha256": digest(np.concatenate([p.nodes.labels.view(np.uint8).ravel(),
                                                          p.nodes.taints.view(np.uint8),
                                                          p.nodes.free.view(np.uint8).ravel(),
                                                          p.nodes.excl.view(np.uint8)]))}
        if cfg != 4:
            rec["assign"] = a.tolist()
        out[str(cfg)] = rec
    with open(os.path.join(ROOT, "tests", "golden", "placements.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
