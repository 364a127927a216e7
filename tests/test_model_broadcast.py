"""tensor_filter framework=pytorch custom=broadcast:<root>: rank 0 reads the
TorchScript file and broadcasts its bytes to every rank at load (comm::Group;
TCP store on CPU, RCCL between GPUs), so all ranks run rank 0's weights even
though each rank's model= points at a different file.  Two processes launched
like torchrun (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT)."""
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = textwrap.dedent(r'''
    import json, os, sys
    sys.path.insert(0, sys.argv[1])
    import numpy as np, torch
    import nnstreamer_amd as nns
    rank = int(os.environ["RANK"])
    torch.manual_seed(100 + rank)  # every rank writes a DIFFERENT model file
    m = torch.nn.Linear(4, 3).eval()
    path = os.path.join(sys.argv[2], f"m{rank}.pt")
    torch.jit.script(m).save(path)
    caps = "other/tensors,format=static,num_tensors=1,dimensions=4,types=float32,framerate=0/1"
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_filter name=f framework=pytorch model={path} "
                         "accelerator=false custom=broadcast:0,broadcast-backend:tcp,broadcast-name:t "
                         "! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).numpy("float32").tolist()))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(np.arange(4, dtype=np.float32), pts=0)
    p.get_by_name("src").end_of_stream()
    assert p.wait(60)[0] == "eos", p.messages()
    group = p.get_by_name("f").get_property("model-broadcast")
    p.stop()
    own = m(torch.arange(4, dtype=torch.float32)).tolist()
    print(json.dumps({"rank": rank, "out": out[0], "own": own, "group": group}), flush=True)
''')


def _free_port():
    from rank_util import free_port

    return free_port()


def test_model_broadcast_two_ranks(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script), ROOT, str(tmp_path)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    res = {}
    for p in procs:
        out, err = p.communicate(timeout=240)
        assert p.returncode == 0, err[-3000:]
        d = json.loads([line for line in out.splitlines() if line.startswith("{")][-1])
        res[d["rank"]] = d
    # both ranks computed with rank 0's weights
    assert not res[1]["group"].startswith("failed"), (res, err[-3000:])
    assert res[0]["out"] == res[1]["out"]
    assert max(abs(a - b) for a, b in zip(res[0]["out"], res[0]["own"])) < 1e-6
    assert max(abs(a - b) for a, b in zip(res[1]["out"], res[1]["own"])) > 1e-3  # rank 1's own file differs
