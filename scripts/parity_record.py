"""Fold the GPU suite's per-comparison parity figures (JSON lines written by
tests/test_gpu_parity.py::_record_elementwise) into one JSON record:

    python scripts/parity_record.py gpurun_out/<tag>/parity_elementwise.jsonl profiles/r06fin_parity_elementwise.json

Per comparison: the scaled contract's worst deviation (parity.compare_maps),
SURVEY §8(d)'s per-element worst and count beyond 1e-5 max(|a|, |b|) over every
compared map entry, the same count over the entries that are not cancellation
entries (weights, covariance diagonals, mean coordinates with |x| >= 1), and
the log-weights' per-element figures.  The summary lists the benched
configurations (the comparisons that assert the non-cancellation count is 0)."""
import json
import sys


def main(src, dst):
    rows = [json.loads(l) for l in open(src) if l.strip()]
    bench = [r for r in rows if r.get("elementwise_asserted")]
    summary = {
        "comparisons": len(rows),
        "elements": sum(r["elements"] for r in rows),
        "elem_beyond": sum(r["elem_beyond"] for r in rows),
        "noncancel_beyond": sum(r["noncancel_beyond"] for r in rows),
        "elem_worst": max((r["elem_worst"] for r in rows), default=0.0),
        "noncancel_worst": max((r["noncancel_worst"] for r in rows), default=0.0),
        "contract_worst": max((r["contract_worst"] for r in rows), default=0.0),
        "benched": {r["label"]: {k: r[k] for k in ("particles", "compared", "elements", "elem_beyond", "elem_worst",
                                                  "noncancel_beyond", "noncancel_worst", "contract_worst",
                                                  "logw_elem_beyond", "logw_elem_worst")} for r in bench},
    }
    json.dump({"summary": summary, "comparisons": rows}, open(dst, "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
