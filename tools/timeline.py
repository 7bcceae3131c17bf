#!/usr/bin/env python3
"""Timeline of the last `--tail` microseconds of a rocprofv3 kernel trace (and, optionally,
its memory-copy trace): start offset, duration, gap to the previous entry's end, queue,
name -- to see what the GPU waits for between kernels."""
import argparse
import csv
import re


def rows(path, kind):
    out = []
    for r in csv.DictReader(open(path)):
        b = int(r.get("Start_Timestamp") or r.get("start_timestamp"))
        e = int(r.get("End_Timestamp") or r.get("end_timestamp"))
        if kind == "k":
            name = re.sub(r"cfdj::\(anonymous namespace\)::|HIP_vector_type<double, 2u>", "",
                          r["Kernel_Name"]).split("(")[0][:48]
            q = r.get("Queue_Id", "?")
        else:
            name = "copy " + r.get("Direction", "")
            q = "c" + r.get("Stream_Id", r.get("Queue_Id", "?"))
        out.append((b, e, q, name))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel_trace")
    ap.add_argument("copy_trace", nargs="?")
    ap.add_argument("--tail", type=float, default=800.0, help="microseconds before the end")
    a = ap.parse_args()
    ev = rows(a.kernel_trace, "k")
    if a.copy_trace:
        ev += rows(a.copy_trace, "c")
    ev.sort()
    end = max(e for _, e, _, _ in ev)
    t0 = end - int(a.tail * 1e3)
    prev_end = None
    for b, e, q, name in ev:
        if b < t0:
            prev_end = max(prev_end or e, e)
            continue
        gap = (b - prev_end) / 1e3 if prev_end else 0.0
        print(f"{(b - t0) / 1e3:9.2f} us  dur {(e - b) / 1e3:8.2f}  gap {gap:7.2f}  q{q:>3}  {name}")
        prev_end = max(prev_end or e, e)


if __name__ == "__main__":
    main()
