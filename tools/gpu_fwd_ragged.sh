for T in 128,128 128,64 64,64; do echo "== $T"; OAC_FWD2_TILE=$T timeout -k 5 60 tools/micro/fwd_micro 1029 13 6 80; done
