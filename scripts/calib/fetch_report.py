"""FETCH_SIZE / WRITE_SIZE per known byte on gfx950 (scripts/calib/calib_fetch.hip).

    python scripts/calib/fetch_report.py <dir> > profiles/fetch_calibration.json

<dir>/fetch and <dir>/write: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of
calib_fetch; <dir>/bytes.csv: its stdout (kernel, known bytes).  Prints, per
calibration kernel, counter bytes / known bytes (FETCH_SIZE and WRITE_SIZE are
reported in KiB)."""
import csv
import glob
import json
import sys


def counter(d, name):
    out = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != name:
                continue
            k = row["Kernel_Name"].split("(")[0]
            out.setdefault(k, []).append(float(row["Counter_Value"]))
    return {k: sum(v) for k, v in out.items()}


def main(d):
    known = {}
    for row in csv.DictReader(open(f"{d}/bytes.csv")):
        known[row["kernel"]] = int(row["bytes"])
    fe = counter(f"{d}/fetch", "FETCH_SIZE")
    wr = counter(f"{d}/write", "WRITE_SIZE")
    res = {}
    for k, b in known.items():
        r = {"known_bytes": b}
        if k in fe:
            r["fetch_bytes"] = fe[k] * 1024
            r["fetch_per_byte"] = round(fe[k] * 1024 / b, 4)
        if k in wr:
            r["write_bytes"] = wr[k] * 1024
            r["write_per_byte"] = round(wr[k] * 1024 / b, 4)
        res[k] = r
    print(json.dumps({"source": "scripts/calib/calib_fetch.hip under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                                "(separate passes), 1 GiB buffers evicted from the Infinity Cache before each kernel",
                      "kernels": res}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
