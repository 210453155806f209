"""Read N > 1 bench lines (the driver's SCALE_rNN.json, BENCH records, or profiles/*scale_rehearsal*.json — any JSON
holding bench.py lines, found wherever they sit) and print the decisions DESIGN.md §11 leaves to the first 8-GPU run,
one line per setting and N, with the medians and spreads they rest on:

* gather direction: the default (pull) column vs `NCCL_AMD_AG_PULL=0` (push);
* release fence: `p2p_fence` on vs off (bitwise-checked columns);
* CU budget: the default channel plan vs `NCCL_MAX_CTAS` 256 / 128 / 64 / 32;
* eager zero-copy vs the staged default;
* size table: `suite.size_table_row.file_line` (ready for an NCCL_AMD_SIZE_TABLE file);
* LL128 class: torn 64-byte lines over a link (`suite.xgmi_probe.store_atomicity`);
* host buffers: the collective on pinned host buffers (`host_staged.direct`) vs the best copy pipeline — whether
  the staged kernel's channel count needs a PCIe-sized plan for host buffers (§11 item 3).

A difference is called only when the two medians differ by more than both columns' spreads (max − min over the
interleaved rounds); otherwise "within spread". usage: python scripts/scale_decisions.py FILE [FILE ...]"""
import json
import sys


def bench_lines(obj):
    """Every bench.py line inside obj (dicts with metric + n_gpus; JSON strings and 'tail' text searched too)."""
    if isinstance(obj, dict):
        if "metric" in obj and "n_gpus" in obj:
            yield obj
            return
        for v in obj.values():
            yield from bench_lines(v)
    elif isinstance(obj, list):
        for v in obj:
            yield from bench_lines(v)
    elif isinstance(obj, str) and '"metric"' in obj:
        for ln in obj.splitlines():
            ln = ln.strip()
            if ln.startswith("{") and '"n_gpus"' in ln:
                try:
                    yield from bench_lines(json.loads(ln))
                except ValueError:
                    pass


def column(runs, env):
    for r in runs:
        if r.get("env") == env:
            return r
    return None


def compare(a, b):
    """'faster' / 'slower' / 'within spread' for column a against column b (medians vs spreads)."""
    if not a or not b:
        return "n/a"
    spread = max(a.get("ms_max", a["ms"]) - a.get("ms_min", a["ms"]), b.get("ms_max", b["ms"]) - b.get("ms_min", b["ms"]))
    d = a["ms"] - b["ms"]
    if abs(d) <= spread:
        return f"within spread ({a['ms']:.4f} vs {b['ms']:.4f} ms, spread {spread:.4f})"
    return f"{'faster' if d < 0 else 'slower'} by {abs(d) / b['ms'] * 100:.1f} % ({a['ms']:.4f} vs {b['ms']:.4f} ms)"


def decisions(line):
    n = line["n_gpus"]
    out = [f"N={n}: value {line.get('value')} GB/s busBW, frac {line.get('roofline', {}).get('frac')} of "
           f"{line.get('roofline', {}).get('peak')} GB/s ({line.get('roofline', {}).get('peak_basis', '')[:60]})"]
    suite = line.get("suite", {})
    runs = suite.get("staged_tuning", {}).get("runs", [])
    dflt = column(runs, "default")
    out.append(f"  gather: pull (default) vs push: {compare(dflt, column(runs, {'NCCL_AMD_AG_PULL': '0'}))}")
    out.append(f"  fence: off vs on: {compare(column(runs, {'NCCL_AMD_P2P_FENCE': '0'}), column(runs, {'NCCL_AMD_P2P_FENCE': '1'}))}"
               f" (default: {line.get('p2p_fence', {}).get('default_fence', 'n/a')})")
    for c in ("256", "128", "64", "32"):
        out.append(f"  channels: default vs NCCL_MAX_CTAS={c}: {compare(dflt, column(runs, {'NCCL_MAX_CTAS': c}))}")
    out.append(f"  eager zero-copy vs default: {compare(column(runs, {'NCCL_AMD_EAGER_REGISTER': '1'}), dflt)}")
    chk = suite.get("ar_fp16_sweep_check")
    if chk:
        bad = {k: v for k, v in chk.items() if not v.startswith("pass")}
        out.append(f"  C4 sweep results: {'every column exact' if not bad else bad}")
    row = suite.get("size_table_row")
    out.append(f"  size table row: {row['file_line'] if row else 'n/a'}")
    atom = suite.get("xgmi_probe", {}).get("store_atomicity")
    if isinstance(atom, dict) and "error" not in atom:
        out.append(f"  LL128 class: store atomicity over a link {json.dumps(atom)[:160]}")
    else:
        out.append("  LL128 class: no link measurement (ranks on one GPU, or the probe did not run)")
    hs = line.get("host_staged", {})
    if "direct" in hs and "pipelined" in hs:
        d, p = hs["direct"], hs["pipelined"]
        out.append(f"  host buffers: direct {d['ms_per_step']} ms ({d['check']}) vs pipelined {p['ms_per_step']} ms at "
                   f"{p['chunks']} chunks ({p['check']}): {d.get('speedup_vs_pipelined')}x")
    return out


def main(paths):
    seen = 0
    for p in paths:
        with open(p) as f:
            data = json.load(f)
        for line in sorted(bench_lines(data), key=lambda d: d["n_gpus"]):
            if line["n_gpus"] < 2:
                continue
            seen += 1
            print("\n".join([f"# {p}"] + decisions(line)))
    if not seen:
        print("no N > 1 bench line found")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
