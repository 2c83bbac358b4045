#!/bin/bash
# conv_bench A/B of a tuning knob on the C2 shapes: bash tools/gpu_conv_ab.sh <tag> <key=value> [shapes...]
set -u
TAG=$1; KV=$2; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
CS=${*:-"8,256,256,46,80,3 8,256,256,92,160,3 8,256,256,23,40,3 8,512,512,23,40,3 8,1024,256,46,80,1 8,256,1024,46,80,1 8,512,2048,23,40,1 8,512,256,92,160,1 8,256,256,92,160,1 8,256,256,92,160,3,2 8,512,512,46,80,3,2"}
timeout -k 10 300 python tools/conv_bench.py $CS > $O/conv_base.jsonl 2> $O/conv.err && \
timeout -k 10 300 python tools/conv_bench.py $KV $CS > $O/conv_ab.jsonl 2>> $O/conv.err; rc=$?
echo "CONV $rc"
python3 - $O <<'PY'
import json, sys
O = sys.argv[1]
a = [json.loads(l) for l in open(O + "/conv_base.jsonl")]
b = [json.loads(l) for l in open(O + "/conv_ab.jsonl")]
for x, y in zip(a, b):
    print(x["shape"], "fwd/dgrad/wgrad us base", x["hip_us"], " ab", y["hip_us"])
PY
exit $rc
