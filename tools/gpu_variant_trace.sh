#!/bin/bash
# Same-box kernel-trace A/B of package variants built by tools/build_variant.sh: the tree's own
# package ("base") and abvar/<tag> for each tag in VARIANTS, bench b32 3 steps, steady-state step.
cd /tmp && export TMPDIR=/tmp && R="${GRAFT_REPO_ROOT:-/root/repo}" && cd "$R"
mkdir -p gpurun_out/vt
for tag in base ${VARIANTS:-noslp}; do
  d="$R"; [ "$tag" != "base" ] && d="$R/abvar/$tag"
  rm -rf "$R/gpurun_out/vt/k_$tag"
  (cd "$d" && timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/vt/k_$tag" -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 2 > "$R/gpurun_out/vt/b_$tag.log" 2>&1) || { tail -5 "$R/gpurun_out/vt/b_$tag.log"; exit 1; }
  echo "$tag $(grep '"metric"' gpurun_out/vt/b_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
  python3 tools/step_kernels.py $(find gpurun_out/vt/k_$tag -name '*kernel_trace.csv') > gpurun_out/vt/t_$tag.txt
  grep -E "step |attn" gpurun_out/vt/t_$tag.txt
done
