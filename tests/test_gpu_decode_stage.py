"""Decoder device stages inside the filter's hipGraph (runtime/fusion.h
DecodeStage): `tensor_filter ! [queue !] tensor_decoder mode=bounding_boxes |
image_segment | pose_estimation` -- the filter appends the decoder's whole device
post-processing (SSD candidates + sort + NMS + raster; DeepLab resize + argmax
+ colour map; PoseNet heatmap argmax + skeleton raster) to its captured
forward and hands out the RGBA frames.  The frames must equal, byte for byte,
the same pipeline with the decoder running its own kernels (absorb-decoder=
false); reference decode paths: tensordec-boundingbox.c:1543-1777,
tensordec-imagesegment.c:328-392, tensordec-pose.c:542-818."""
import os

import pytest

pytestmark = pytest.mark.gpu


def _files(workdir):
    from nnstreamer_amd.models.posenet import write_pose_labels
    from nnstreamer_amd.models.ssd import write_box_priors, write_coco_labels

    return dict(coco=write_coco_labels(os.path.join(workdir, "coco_st.txt")),
                priors=write_box_priors(os.path.join(workdir, "priors_st.txt")),
                pose=write_pose_labels(os.path.join(workdir, "pose17_st.txt")))


CASES = {
    "ssd": (300, "ssd_fused_fp32", "typecast:float32,add:-127.5,div:127.5",
            "tensor_decoder name=dec mode=bounding_boxes option1=mobilenet-ssd option2={coco} option3={priors} "
            "option4=300:300 option5=300:300"),
    "deeplab": (513, "deeplab_fused_lowres_fp32", "typecast:float32,div:255.0",
                "tensor_decoder name=dec mode=image_segment option1=tflite-deeplab option3=513:513"),
    "posenet": (257, "posenet_fused_fp32", "typecast:float32,add:-127.5,div:127.5",
                "tensor_decoder name=dec mode=pose_estimation option1=640:480 option2=257:257 option3={pose} "
                "option4=heatmap-offset"),
}


def _run(nns, workdir, case, B, absorb, graph, queue, lanes=0):
    from nnstreamer_amd.models.export import export

    S, model_name, norm, dec = CASES[case]
    model = export(model_name, os.path.join(workdir, f"{model_name}_st.pt"), layout="nhwc")
    q = "queue max-size-buffers=2 ! " if queue else ""
    desc = (f"videotestsrc num-buffers={3 * B} pattern=snow pool-size={3 * B} "
            f"! video/x-raw,format=RGB,width={S},height={S},framerate=30/1 "
            f"! tensor_converter frames-per-tensor={B} device=0 ! tensor_transform mode=arithmetic option={norm} "
            f"! tensor_filter name=f framework=pytorch model={model} input=3:{S}:{S}:{B} inputtype=float32 "
            f"accelerator=true:gpu device=0 custom=hipgraph:{'true' if graph else 'false'}"
            f"{f',lanes:{lanes}' if lanes else ''} "
            f"absorb-decoder={'true' if absorb else 'false'} ! {q}{dec.format(**_files(workdir))} "
            "! tensor_sink name=sink")
    p = nns.parse_launch(desc)
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(bytes(b.memory(0).bytes())))
    p.run(timeout=300)
    info = (p.get_by_name("f").get_property("absorbed-decoder"), p.get_by_name("dec").get_property("stage-by"))
    p.stop()
    return out, info


@pytest.mark.parametrize("case,B,graph,queue", [("ssd", 4, True, True), ("ssd", 1, True, False),
                                                ("deeplab", 2, True, True), ("posenet", 4, True, True),
                                                ("posenet", 2, False, True)])
def test_decoder_stage_in_graph_matches_own_kernels(nns, workdir, case, B, graph, queue):
    got, info = _run(nns, workdir, case, B, True, graph, queue)
    ref, info_ref = _run(nns, workdir, case, B, False, graph, queue)
    assert info == ("dec", "f"), info
    assert info_ref == ("", ""), info_ref
    assert len(got) == len(ref) == 3 * B
    assert got == ref
    if case != "ssd":  # (random-init SSD may detect nothing)
        assert any(any(x) for x in got[:4])  # something was drawn


@pytest.mark.parametrize("case", ["ssd", "posenet", "deeplab"])
def test_decoder_stage_with_replay_lanes_asked(nns, workdir, case):
    """custom=lanes:3 with a decoder stage absorbed.  SSD's and PoseNet's stages
    keep scratch in the stage object, so the filter replays on one lane
    (lane_count); DeepLab's (resize + argmax + colour map) writes only its output
    frames (DecodeStage::lane_safe), so its graphs replay on three lanes at once.
    Either way the frames equal, byte for byte, the decoder running its own
    kernels"""
    got, info = _run(nns, workdir, case, 4, True, True, True, lanes=3)
    ref, _ = _run(nns, workdir, case, 4, False, True, True, lanes=3)
    assert info == ("dec", "f"), info
    assert len(got) == len(ref) == 12
    assert got == ref


def test_decoder_option_change_retakes_stage(nns, workdir):
    """A decoder option set while playing (pose_estimation option4
    heatmap-offset -> heatmap-only) after the filter captured the decoder's stage
    in its graph: the stage goes stale (tensor_decoder.cc InstanceStage::revoke),
    the filter re-takes it and re-captures, and the later frames equal a run
    that had the new option from the start -- no frozen options, no freed
    decoder instance under a live graph."""
    from nnstreamer_amd.models.export import export

    S, model_name, norm, dec = CASES["posenet"]
    model = export(model_name, os.path.join(workdir, f"{model_name}_opt.pt"), layout="nhwc")
    B, nb = 2, 8

    def run(option4, switch_after=None):
        d = dec.format(**_files(workdir)).replace("option4=heatmap-offset", f"option4={option4}")
        desc = (f"videotestsrc num-buffers={nb * B} pattern=snow pool-size={nb * B} "
                f"! video/x-raw,format=RGB,width={S},height={S},framerate=30/1 "
                f"! tensor_converter frames-per-tensor={B} device=0 ! tensor_transform mode=arithmetic option={norm} "
                f"! tensor_filter name=f framework=pytorch model={model} input=3:{S}:{S}:{B} inputtype=float32 "
                "accelerator=true:gpu device=0 custom=hipgraph:true ! queue max-size-buffers=2 "
                f"! {d} ! tensor_sink name=sink")
        p = nns.parse_launch(desc)
        out = []

        def on(b):
            out.append(bytes(b.memory(0).bytes()))
            if switch_after is not None and len(out) == switch_after:
                p.get_by_name("dec").set_property("option4", "heatmap-only")

        p.get_by_name("sink").connect("new-data", on)
        p.run(timeout=300)
        info = p.get_by_name("f").get_property("absorbed-decoder")
        p.stop()
        return out, info

    switched, info = run("heatmap-offset", switch_after=2)
    ref, _ = run("heatmap-only")
    off, _ = run("heatmap-offset")
    assert info == "dec"
    assert len(switched) == len(ref) == nb * B
    assert switched[-4:] == ref[-4:]      # the last two batches ran the new option
    assert switched[:2] == off[:2]        # the first frames ran the old one
    assert ref != off                     # (the option changes the frames)
