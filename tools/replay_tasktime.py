"""Spread of the replay generator's task times (a MPSS_REPLAY_TASKTIME build's "tasktime" lines:
task, sub-window origin, pixels, camera hits, wall time in 100 MHz ticks), per launch.

    python tools/replay_tasktime.py LOG
"""
import sys

import numpy as np


def main(path):
    rows = []
    for line in open(path, errors="replace"):
        if line.startswith("tasktime "):
            f = line.split()
            if len(f) == 7:
                rows.append([int(x) for x in f[1:]])
    a = np.array(rows, dtype=np.int64)
    if len(a) == 0:
        print("no tasktime lines")
        return
    # every task prints once per launch: the last launch is the last (number of distinct tasks) lines
    n = len(np.unique(a[:, 0]))
    last = a[-n:]
    us = last[:, 5] / 100.0
    hits = last[:, 4]
    pix = last[:, 3]
    print("tasks %d (of %d lines), time us: median %.0f p90 %.0f p99 %.0f max %.0f" %
          (len(last), len(a), np.median(us), np.percentile(us, 90), np.percentile(us, 99), us.max()))
    nohit = hits == 0
    if nohit.any():
        print("tasks with no camera hit: %d, time us median %.0f max %.0f" % (nohit.sum(), np.median(us[nohit]), us[nohit].max()))
    if (~nohit).any():
        print("tasks with hits: %d, time us median %.0f max %.0f; hits per pixel median %.1f" %
              (( ~nohit).sum(), np.median(us[~nohit]), us[~nohit].max(), np.median(hits[~nohit] / np.maximum(pix[~nohit], 1))))
    order = np.argsort(-us)[:12]
    print("slowest: task x0 y0 pixels hits us")
    for i in order:
        print("  %5d %5d %5d %4d %6d %7.0f" % (last[i, 0], last[i, 1], last[i, 2], pix[i], hits[i], us[i]))
    c = np.corrcoef(hits / np.maximum(pix, 1), us)[0, 1]
    print("correlation(time, hits per pixel) = %.3f" % c)


if __name__ == "__main__":
    main(sys.argv[1])
