"""Per-thread CPU time of a running process over an interval (diagnostics: which threads of a
bench run are busy).  python tools/thread_cpu.py PID [seconds]"""
import os
import sys
import time


def snap(pid):
    out = {}
    for tid in os.listdir(f"/proc/{pid}/task"):
        try:
            st = open(f"/proc/{pid}/task/{tid}/stat").read()
            comm = st[st.index("(") + 1:st.rindex(")")]
            f = st[st.rindex(")") + 2:].split()
            out[tid] = (comm, int(f[11]) + int(f[12]))
        except OSError:
            pass
    return out


pid, dt = int(sys.argv[1]), float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
a = snap(pid)
time.sleep(dt)
b = snap(pid)
hz = os.sysconf("SC_CLK_TCK")
agg = {}
for tid, (comm, t) in b.items():
    d = (t - a.get(tid, (comm, t))[1]) / hz / dt
    agg.setdefault(comm, [0.0, 0])
    agg[comm][0] += d
    agg[comm][1] += 1
for comm, (cores, n) in sorted(agg.items(), key=lambda x: -x[1][0]):
    print(f"{comm:20s} threads {n:4d} cores {cores:6.2f}")
per = sorted(((b[t][1] - a.get(t, b[t])[1]) / hz / dt, t) for t in b)
busy = [c for c, _ in per if c > 0.05]
print(f"threads above 5% of a core: {len(busy)}; top: " + ", ".join(f"{c:.2f}" for c, _ in per[::-1][:12]))
