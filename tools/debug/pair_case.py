"""Debug: the golden f32 + [4, 4] case through the word-pair path."""
import os, sys
import numpy as np
REPO = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "simd-radix-sort_amd", "python"))
import srs_amd
from srs_testlib import golden_manifest, golden_arrays, stable_reference
os.environ.setdefault("SRS_TRACE_LEVELS", "1")
for c in golden_manifest()["cases"]:
    if c["family"] == "large" and c["key_kind"] == 8 and c["payload_sizes"] == [4, 4]:
        ins, outs = golden_arrays(c)
        cols = [a.copy() for a in ins]
        srs_amd.sort_thresh(c["thresh"], cols[0], *cols[1:], up=bool(c["up"]))
        bad = [i for i in range(3) if not np.array_equal(cols[i].view(np.uint8), outs[i].view(np.uint8))]
        print(c["dist"], c["n"], c["up"], "bad cols", bad, flush=True)
        for i in bad:
            d = np.nonzero(cols[i].view(np.uint32) != outs[i].view(np.uint32))[0]
            print("  col", i, "ndiff", len(d), "first", d[:10], "got", cols[i].view(np.uint32)[d[:4]],
                  "want", outs[i].view(np.uint32)[d[:4]], flush=True)
