"""Timeline of one pipelined headline step from a rocprofv3 kernel-trace CSV
(tools/gpu_r06_trace.sh): every kernel between two fused-stem starts, its
queue (conv stream / encoder stream), start/end relative to the stem and
duration, plus the conv stream's idle time in the step.
    python tools/pipe_timeline.py gpurun_out/prof6_pipe/run_kernel_trace.csv [step-from-end]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    stems = [i for i, r in enumerate(rows) if "stem224_fused" in r["Kernel_Name"]]
    a, b = stems[-back - 1], stems[-back]
    t0 = int(rows[a]["Start_Timestamp"])
    q_conv = rows[a]["Queue_Id"]
    busy_end, idle = None, 0.0
    for r in rows[a:b + 1]:
        s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
        q = r["Queue_Id"]
        if q == q_conv:
            if busy_end is not None and s > busy_end:
                idle += s - busy_end
            busy_end = e if busy_end is None else max(busy_end, e)
        name = r["Kernel_Name"].replace("void fac::", "")[:38]
        print(f"{s:9.2f} {e:9.2f} {e - s:8.2f}  {'conv' if q == q_conv else 'tail'}  {name}")
    step = (int(rows[b]["Start_Timestamp"]) - t0) / 1e3
    print(f"step {step:.1f} us, conv-stream idle {idle:.1f} us")


if __name__ == "__main__":
    main()
