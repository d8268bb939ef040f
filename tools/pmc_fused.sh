set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pf
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pf/fetch -o p -- python3 tools/fused_check.py 200 > gpurun_out/pf/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pf/write -o p -- python3 tools/fused_check.py 200 > gpurun_out/pf/write.log 2>&1
python3 - <<'PY'
import csv, glob, collections
for tag in ('fetch', 'write'):
    acc = collections.defaultdict(list)
    for f in glob.glob(f'gpurun_out/pf/{tag}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r['Kernel_Name'].split('(')[0][-60:]].append(float(r['Counter_Value']))
    for k, v in acc.items():
        if 'rds' in k or 'doppler' in k or 'range' in k or 'finish' in k:
            print(tag, k, len(v), [round(x / 1024, 1) for x in v[:8]], 'MiB')
PY
