# adaptive rounds (reference defaults aTolerance 0.05, aBatch 10): round-length knobs (env, host side)
export CFGS="ad --adaptive"
export ARMS="base RT_AMD_ADAPT_GROW=3
f20 RT_AMD_ADAPT_FIRST=20
f30 RT_AMD_ADAPT_FIRST=30
f40 RT_AMD_ADAPT_FIRST=40
g4 RT_AMD_ADAPT_GROW=4
g6 RT_AMD_ADAPT_GROW=6
f20g6 RT_AMD_ADAPT_FIRST=20 RT_AMD_ADAPT_GROW=6
j300 RT_AMD_ADAPT_JUMP=300"
bash tools/gpu_run.sh r05_l ab || exit $?
