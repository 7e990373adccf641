# source me: build_variant NAME SED_EXPR [FILE]  -- library variant (SED_EXPR applied to FILE,
# default n4.hip) built into scratch_libs/NAME.so for A/B runs (scripts/gpu_ab.sh, VH_LIB_PATH).
build_variant ()
{
    local f=${3:-n4.hip}
    rm -rf /tmp/vbroot && mkdir -p /tmp/vbroot/vent_analysis_amd && cp -r include /tmp/vbroot/ && cp -r vent_analysis_amd/csrc /tmp/vbroot/vent_analysis_amd/ && rm -rf /tmp/vbroot/vent_analysis_amd/csrc/build && ( cd /tmp/vbroot/vent_analysis_amd/csrc && sed -i "$2" $f && make -j8 OUT=/root/repo/scratch_libs/$1.so > /dev/null 2>&1 ) && echo built $1
}
