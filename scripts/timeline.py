"""Where a bench step's wall time goes, from a rocprofv3 kernel trace (gpu_round.sh's kt/ directory):

  * per batch boundary (k_logmel launches): encoder-stream busy time, decoder busy time, time with both busy,
    time with neither busy (host or dependency gaps);
  * decode steps (k_select_final* to k_select_final*) with the encoder active vs idle: span and kernel-time sum,
    so the in-context inflation of a step splits into longer kernels vs longer gaps.

    python scripts/timeline.py gpurun_out/<tag>
"""
import bisect
import csv
import glob
import sys

ENC = {"k_gemm_big", "k_gemm_8p", "k_gemm_8pp", "k_gemm_h", "k_gemm_ns", "k_gemm_tile", "k_gemm_mx", "k_gemm_8p_mx",
       "k_attn_enc2", "k_attn_enc3", "k_attn_encoder", "k_layernorm", "k_layernorm_mx", "k_im2col_conv1",
       "k_im2col_conv2", "k_logmel", "k_logmel_finalize"}


def short(name: str) -> str:
    return name.replace("void ", "").split("(")[0].split("<")[0].strip()


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def covered(u, lo, hi):
    return sum(min(e, hi) - max(s, lo) for s, e in u if e > lo and s < hi)


def inter(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def main(root):
    rows = []
    for f in glob.glob(root + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    enc = union([(s, e) for s, e, n in rows if n in ENC])
    dec_rows = [(s, e, n) for s, e, n in rows if n not in ENC and n.startswith("k_")]
    dec = union([(s, e) for s, e, _ in dec_rows])
    both = inter(enc, dec)
    marks = [s for s, _, n in rows if n == "k_logmel"] + [rows[-1][1]]
    print(f"{'batch':>5s} {'span_ms':>8s} {'enc_ms':>7s} {'dec_ms':>7s} {'both_ms':>7s} {'idle_ms':>7s}")
    for i in range(len(marks) - 1):
        lo, hi = marks[i], marks[i + 1]
        ce, cd, cb = covered(enc, lo, hi), covered(dec, lo, hi), covered(both, lo, hi)
        idle = (hi - lo) - (ce + cd - cb)
        print(f"{i:5d} {(hi - lo) / 1e6:8.2f} {ce / 1e6:7.2f} {cd / 1e6:7.2f} {cb / 1e6:7.2f} {idle / 1e6:7.2f}")
    starts = [x[0] for x in enc]

    def enc_active(t):
        k = bisect.bisect_right(starts, t) - 1
        return k >= 0 and enc[k][1] >= t

    steps, cur = [], []
    for r in dec_rows:
        cur.append(r)
        if r[2].startswith("k_select_final"):
            steps.append(cur)
            cur = []
    agg = {}
    for label, want in (("encoder active", True), ("encoder idle", False)):
        sel = [s for s in steps[1:] if enc_active((s[0][0] + s[-1][1]) // 2) == want and len(s) > 20]
        if not sel:
            print(f"decode steps with {label}: none")
            continue
        span = sorted((s[-1][1] - s[0][0]) / 1e3 for s in sel)
        ksum = sorted(sum(e - b for b, e, _ in s) / 1e3 for s in sel)
        print(f"decode steps with {label}: n={len(sel)} span median {span[len(span) // 2]:.1f} us "
              f"(kernels {ksum[len(ksum) // 2]:.1f} us, {len(sel[0])} launches)")
        for s in sel:
            for b, e, n in s:
                agg.setdefault((n, want), []).append((e - b) / 1e3)
    print(f"{'decoder kernel':28s} {'n_act':>6s} {'idle_us':>8s} {'active_us':>9s}")
    for n in sorted({n for n, _ in agg}):
        i, a = sorted(agg.get((n, False), [0])), sorted(agg.get((n, True), [0]))
        print(f"{n:28s} {len(agg.get((n, True), [])):6d} {i[len(i) // 2]:8.2f} {a[len(a) // 2]:9.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
