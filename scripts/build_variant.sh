build_variant () 
{ 
    rm -rf /tmp/vbroot && mkdir -p /tmp/vbroot/vent_analysis_amd && cp -r include /tmp/vbroot/ && cp -r vent_analysis_amd/csrc /tmp/vbroot/vent_analysis_amd/ && rm -rf /tmp/vbroot/vent_analysis_amd/csrc/build && ( cd /tmp/vbroot/vent_analysis_amd/csrc && sed -i "$2" n4.hip && make -j8 OUT=/root/repo/scratch_libs/$1.so > /dev/null 2>&1 ) && echo built $1
}
