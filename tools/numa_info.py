"""Host NUMA layout and the NUMA node of each visible GPU (sysfs), as one
JSON line.  No GPU call: reads /sys only (tools/, not a test)."""
import glob
import json
import os


def main():
    nodes = {}
    for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
        try:
            nodes[os.path.basename(d)] = open(os.path.join(d, "cpulist")).read().strip()
        except OSError:
            pass
    gpus = []
    for dev in sorted(glob.glob("/sys/bus/pci/devices/*")):
        try:
            vendor = open(os.path.join(dev, "vendor")).read().strip()
            cls = open(os.path.join(dev, "class")).read().strip()
        except OSError:
            continue
        if vendor == "0x1002" and cls.startswith(("0x0380", "0x0300", "0x1200")):
            try:
                numa = open(os.path.join(dev, "numa_node")).read().strip()
            except OSError:
                numa = None
            gpus.append({"pci": os.path.basename(dev), "class": cls, "numa_node": numa})
    print(json.dumps({"nodes": nodes, "amd_gpus": gpus,
                      "visible": {k: os.environ.get(k) for k in
                                  ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                   "CUDA_VISIBLE_DEVICES")},
                      "affinity_cpus": len(os.sched_getaffinity(0))}))


if __name__ == "__main__":
    main()
