"""Folds the per-check margin lines that tests/helpers.close appends to $DGS_MARGINS into one
JSON document (profiles/rNN_margins.json): per test, per check, the margin max|got - ref| / bound
(< 1 passes) with the tolerance it was measured against, plus the worst checks overall.

    python tools/margins_summary.py gpurun_out/margins.jsonl > profiles/r04_margins.json
"""
import json
import sys


def main(path):
    rows = [json.loads(line) for line in open(path) if line.strip()]
    by_test = {}
    for r in rows:
        key = r["what"]
        t = by_test.setdefault(r["test"], {})
        old = t.get(key)
        if old is None or r["margin"] > old["margin"]:
            t[key] = {"margin": round(r["margin"], 4), "rtol": r["rtol"], "atol_frac": r["atol_frac"],
                      "n": r["n"]}
    allm = [(m["margin"], test, what, m["atol_frac"]) for test, t in by_test.items() for what, m in t.items()]
    allm.sort(reverse=True)
    # bracketed records are informational: the reference's own spreads ("[reference serial order
    # vs exact]", "[reference fmad vs no-contract]") and the plain-bound view of stated-bound checks
    flat = [f for f in allm if "[" not in f[2]]
    info = [f for f in allm if "[" in f[2]]
    grad = [f for f in flat if "/d" in f[2] or f[2].startswith("d")]
    doc = {
        "source": path,
        "checks": len(rows),
        "tests": len(by_test),
        "failing": [{"margin": m, "test": t, "what": w, "atol_frac": a} for m, t, w, a in flat if m > 1.0],
        "worst": [{"margin": m, "test": t, "what": w, "atol_frac": a} for m, t, w, a in flat[:25]],
        "worst_gradients_at_atol_1e-6": [{"margin": m, "test": t, "what": w}
                                         for m, t, w, a in grad if a == 1e-6][:25],
        "reference_spreads_and_plain_bounds_worst": [{"margin": m, "test": t, "what": w} for m, t, w, a in info[:40]],
        "by_test": by_test,
    }
    json.dump(doc, sys.stdout, indent=1)
    sys.stdout.write("\n")


if __name__ == "__main__":
    main(sys.argv[1])
