# Same-box A/B of the tree's conv1s against an experiment build ab/<name> (tools/build_variant.sh), both orders:
# step time and the per-shape conv1s times.  usage: bash tools/ab_conv1s_variant.sh <name>
V=$1
show() {
  python3 -c "
import json
for v in ('$1', '$2'):
    d = json.load(open(f'gpurun_out/var/{v}.json'))
    print(v, round(d['ms_per_step'], 2), {k.split('@')[0][14:] + '@' + k.split('@')[1]: x['avg_us'] for k, x in d['shapes'].items() if 'conv1s' in k})
"
}
BENCH_ARGS="--n-timesteps 10" bash tools/ab_variants.sh tree $V > /dev/null || exit 1
show tree $V
BENCH_ARGS="--n-timesteps 10" bash tools/ab_variants.sh $V tree > /dev/null || exit 1
show $V tree
