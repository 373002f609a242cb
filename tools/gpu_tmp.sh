AB_ROWS=40 bash tools/ab_variants.sh wpf0 tree wpf0 tree > gpurun_out/ab_wpf.txt 2>&1; rc=$?; grep -E "variant|ms/step|attn_kv" gpurun_out/ab_wpf.txt; exit $rc
