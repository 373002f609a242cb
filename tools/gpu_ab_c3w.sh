AB_ROWS=12 bash tools/ab_variants.sh tree xd3 xd4 && GRADTTS_LIB=$PWD/ab/st/libgradtts.so timeout -k 10 120 python3 tools/diag_c3w_stamps.py
