"""Per-kernel timeline of the last timed step in a rocprofv3 kernel-trace csv
directory: start/end in µs from the step's first phip kernel, per stream
(queue).  The last step = the kernels after the last k_resolve / k_classify
launch that opens a step."""
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append(r)
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
opener = sys.argv[2] if len(sys.argv) > 2 else "k_resolve"
starts = [i for i, r in enumerate(rows) if opener in r["Kernel_Name"] and "miss" not in r["Kernel_Name"]]
if not starts:
    sys.exit("no %s in trace" % opener)
i0 = starts[-1]
t0 = int(rows[i0]["Start_Timestamp"])
# back up to the step's counter reset (kernels just before the opener)
print("%-38s %6s %9s %9s %8s" % ("kernel", "queue", "start_us", "end_us", "dur_us"))
for r in rows[max(0, i0 - 4):]:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("phip::", "")
    if "rocprim" in name:
        name = "rocprim:" + name.split("::")[-1][:28]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%-38s %6s %9.1f %9.1f %8.1f" % (name[:38], r.get("Queue_Id", r.get("Stream_Id", "?")),
                                         (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
