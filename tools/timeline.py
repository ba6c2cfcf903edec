#!/usr/bin/env python3
"""Kernel timeline (start, end, duration in ms from the first dispatch) of a rocprofv3
kernel_trace.csv; blit kernels included. usage: timeline.py kernel_trace.csv [t_from_ms]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
t0 = min(int(r["Start_Timestamp"]) for r in rows)
tf = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    if s >= tf and "vectorized" not in r["Kernel_Name"]:
        print(f"{r['Kernel_Name'][:34]:34s} q{r['Queue_Id']} {s:9.2f} {e:9.2f} {e - s:8.2f}")
