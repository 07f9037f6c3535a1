# round 6, call b: k_tconv_chain patch-load policy A/B (config 5): sc1 (product) vs sc0 (round 5) vs nt vs sc0 sc1
LIBS="'' _p0 _pnt _pss" REPS=2 ARGS="--config 5 --no-cpu-baseline" bash scripts/gpu_ab.sh
