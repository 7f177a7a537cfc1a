R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/romab; mkdir -p $O
for w in config3 config2; do for r in ${ROMS:-d049f8b 3d69517 new}; do
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --workload $w --rom tmp_roms/pk_$r.gb > $O/${w}_$r.json 2>>$O/err.log || exit $?
done; done
