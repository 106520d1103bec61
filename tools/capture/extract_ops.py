#!/usr/bin/env python3
"""Extract the capture's stream/event ops from an AMD_LOG_LEVEL=4 log (tools/capture/replay.cpp input):
from hipStreamBeginCapture to hipStreamEndCapture, in log order."""
import re
import sys

pat = re.compile(r"\b(hipStreamBeginCapture|hipEventRecord|hipStreamWaitEvent|hipMemcpyAsync|hipLaunchKernel|"
                 r"hipStreamEndCapture) \( ([^)]*)\)")
on = False
for line in open(sys.argv[1], errors="replace"):
    m = pat.search(line)
    if not m or "Returned" in line:
        continue
    fn, args = m.group(1), [x.strip() for x in m.group(2).split(",")]
    if fn == "hipStreamBeginCapture":
        on = True
        print("B", args[0])
    elif not on:
        continue
    elif fn == "hipEventRecord":
        print("R", args[0], args[1])
    elif fn == "hipStreamWaitEvent":
        print("W", args[0], args[1])
    elif fn == "hipMemcpyAsync":
        print("M", args[-1])
    elif fn == "hipLaunchKernel":
        print("K", args[-1])
    elif fn == "hipStreamEndCapture":
        print("E", args[0])
        break
