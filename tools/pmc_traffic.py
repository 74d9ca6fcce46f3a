"""Per-launch HBM traffic of a kernel from rocprofv3 PMC runs (separate FETCH_SIZE / WRITE_SIZE passes).

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports half the
bytes of wide (16 B/lane) coalesced reads -> doubled; WRITE_SIZE is exact for
16-B stores. Both counters are in KiB.

    python tools/pmc_traffic.py <fetch_csv> <write_csv> <kernel-substring[+kernel2...]> [out.json] [--largest]

--largest keeps, per counter, the largest launch instead of the median (for a
command that launches the same kernel at several sizes, e.g. the two
GraphSAGE layers, where the bench's roofline names the largest).

--steps N sums every matching launch and divides by N: for a step that launches one
kernel more than once (the XCD-sliced hub SpMM runs spmm_csr_kernel for both passes);
run the bench with --no-layer so that only the N = warmup + steps aggregation steps launch
those kernels.
"""
import csv
import json
import statistics
import sys


STEPS = None


def per_launch(path, counter, kernel, largest=False):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel!r} in {path}")
    if STEPS:
        return sum(vals) / STEPS, len(vals)
    return (max(vals) if largest else statistics.median(vals)), len(vals)


def main():
    global STEPS
    largest = "--largest" in sys.argv
    argv = [a for a in sys.argv if a != "--largest"]
    if "--steps" in argv:
        i = argv.index("--steps")
        STEPS = int(argv[i + 1])
        del argv[i:i + 2]
    fetch_csv, write_csv, kernel = argv[1:4]
    # "a+b+c": one logical launch made of several kernels -> sum of their per-launch values
    parts = kernel.split("+")
    fw = [(per_launch(fetch_csv, "FETCH_SIZE", k, largest), per_launch(write_csv, "WRITE_SIZE", k, largest))
          for k in parts]
    f = sum(a[0] for a, _ in fw)
    w = sum(b[0] for _, b in fw)
    nf = [a[1] for a, _ in fw]
    nw = [b[1] for _, b in fw]
    res = {"kernel": kernel, "fetch_kib_raw": f, "write_kib": w, "launches": [nf, nw],
           "fetch_bytes_corrected": 2 * f * 1024, "write_bytes": w * 1024,
           "traffic_bytes": (2 * f + w) * 1024,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read halving), WRITE_SIZE exact; KiB->B"}
    if STEPS:
        res["selection"] = f"sum of all launches / {STEPS} steps"
    if largest:
        res["selection"] = "largest launch"
    out = json.dumps(res, indent=1)
    if len(argv) > 4:
        open(argv[4], "w").write(out + "\n")
    print(out)


if __name__ == "__main__":
    main()
