cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cf -o k --output-format csv -- python3 bench.py --no-cpu --no-file --steps 5 > $O/cf.json 2> $O/cf.err || { tail $O/cf.err; exit 1; }
NLDSC_COUNT_FREE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ct -o k --output-format csv -- python3 bench.py --no-cpu --no-file --steps 5 > $O/ct.json 2> $O/ct.err || { tail $O/ct.err; exit 1; }
find $O/prof_cf -name "*kernel_stats.csv" -exec cp {} $O/stats_cf.csv \;
find $O/prof_ct -name "*kernel_stats.csv" -exec cp {} $O/stats_ct.csv \;
cut -d, -f1-8 $O/stats_cf.csv | head -14; echo; cut -d, -f1-8 $O/stats_ct.csv | head -14
