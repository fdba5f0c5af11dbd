# where the launch tail goes: per-wave start / dry / end clocks (variant wprobe, RT_WAVE_PROBE=1)
mkdir -p gpurun_out/r05_v
RT_AMD_VARIANT=wprobe timeout -k 10 300 python tools/wave_probe.py cornell spheres rain > gpurun_out/r05_v/wave_probe.log 2>&1 || exit $?
