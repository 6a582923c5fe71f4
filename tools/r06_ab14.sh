# round 6: wider channel chunks for the 3x3 MTW-1 DMA dwpw (ZARU_HIP_DFKC=32 / 64) on the face networks
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
LAYER_MODELS="face_landmark:256 face_detection_short_range:256" bash tools/gpu_layers.sh r06r_l "" "ZARU_HIP_DFKC=32" "ZARU_HIP_DFKC=64"
