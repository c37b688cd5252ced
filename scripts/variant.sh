# Sourced by the A/B scripts.  A variant is a space-separated list of tokens:
# NAME=value tokens whose NAME is upper case (RT_TRACE_LIB=librt_trace_base.so for a
# library build, RT_STATS=1) go to the environment; everything else is passed to
# bench.py (--opt XcdGroup=off --opt LanesPerPixel=16: rt_device_options, which the
# library takes through the C-ABI only).  "default" is the empty variant.
split_variant() {
  VENV=(); VARGS=()
  local prev=""
  for tok in $1; do
    if [ "$tok" = default ]; then :
    elif [ "$prev" != "--opt" ] && [[ "$tok" =~ ^[A-Z_][A-Z0-9_]*= ]]; then VENV+=("$tok")
    else VARGS+=("$tok"); fi
    prev=$tok
  done
}
