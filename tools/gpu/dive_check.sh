# the N = 4 continuation paths' GPU tests, a bench line and the chain
# diagnostics of syn4x200 (tools/gpu/libpastar_gpu_phases.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "continuation or score_bit_exact or random or cli" 2>&1 | tail -3 || exit 1
for i in 1 2; do
timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-north-star --no-sub-records > gpurun_out/sw.json || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); print('ms/step %.3f loop %.3f exp %d steps %.1f launch %.1f us ok %s' % (d['ms_per_step'], d['search_loop_s']*1e3, d['expansions_per_search'], d['steps_per_search'], d['roofline']['avg_launch_us'], d['score_ok']))"
done
[ -f tools/gpu/libpastar_gpu_phases.so ] && bash tools/gpu/phases.sh syn4x200_s1 3 | tail -6
