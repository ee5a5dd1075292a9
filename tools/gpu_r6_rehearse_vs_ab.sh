cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6why; mkdir -p $O
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu --no-file --steps 20 --rehearse 0/8 > $O/reh$i.json 2> $O/reh.err || exit 1
python3 -c "import json; d=json.loads(open('$O/reh$i.json').read().strip().splitlines()[-1]); print('rehearse', round(d['ms_per_step'],4), d['stages_ms'])"
timeout -k 10 300 python tools/ab_libs.py --libs new=nldsc_amd/libnldsc_amd.so --workload c3r0of8 --runs 20 > $O/ab$i.json 2> $O/ab.err || exit 1
python3 -c "
import json; d=json.loads(open('$O/ab$i.json').read())['ab']
for wl,v in d.items():
    for k,x in v.items(): print('ab', wl, k, round(x['band_ms_median'],4), round(x['total_ms_median'],4))"
done
