#!/bin/bash
# gpurun wrapper: run "$1" with timeout $2 (s), print the verdict line and the status
T=${2:-600}
timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout $T -- "$1" > /tmp/g_last.txt 2>&1
python3 -c "
import json; d=json.load(open('/root/repo/gpurun_out/.last_call.json'))
print('STATUS', d['status'], 'rc', d['rc'], 'run_s', round(d.get('run_s') or 0), 'left', d.get('gpu_minutes_left'), (d.get('msg') or '')[:160])"
