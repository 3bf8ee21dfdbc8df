"""Diagnose 2-worker (gloo, both on cuda:0) vs 1-process ASRTask.main training: per-epoch
train/valid losses with one global batch per epoch (batch_size 16), Adam eps 1 (update ~ lr*g)
and default eps."""
import os, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "espnet-1_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch, yaml
from test_task_gpu import _corpus
from espnet_amd.tasks.asr import ASRTask

def main():
    tmp = __import__("pathlib").Path(tempfile.mkdtemp())
    (tmp / "tr").mkdir(); (tmp / "dv").mkdir()
    tr = _corpus(tmp / "tr", 16); dv = _corpus(tmp / "dv", 4, seed=1)
    for d_, seed in ((tr, 3), (dv, 4)):
        rng = np.random.RandomState(seed); lines = []
        for ln in (d_ / "speech_shape").read_text().split("\n"):
            if ln:
                utt, shp = ln.split(); f = d_ / f"{utt}.npy"
                np.save(f, rng.randn(*[int(x) for x in shp.split(",")]).astype(np.float32)); lines.append(f"{utt} {f}")
        (d_ / "feats.scp").write_text("\n".join(lines) + "\n")
    V = 30
    (tmp / "tokens.txt").write_text("\n".join(["<blank>", "<unk>"] + [f"c{i}" for i in range(V - 3)] + ["<sos/eos>"]) + "\n")
    for bs, eps in ((16, 1e-8), (16, 1.0), (4, 1.0)):
        conf = dict(encoder="transformer",
                    encoder_conf=dict(output_size=64, attention_heads=4, linear_units=256, num_blocks=2,
                                      dropout_rate=0.0, positional_dropout_rate=0.0, attention_dropout_rate=0.0),
                    decoder="transformer",
                    decoder_conf=dict(attention_heads=4, linear_units=256, num_blocks=2, dropout_rate=0.0,
                                      positional_dropout_rate=0.0, self_attention_dropout_rate=0.0,
                                      src_attention_dropout_rate=0.0),
                    model_conf=dict(ctc_weight=0.3, lsm_weight=0.1, length_normalized_loss=False),
                    optim="adam", optim_conf=dict(lr=0.002, eps=eps), scheduler="warmuplr",
                    scheduler_conf=dict(warmup_steps=10), batch_type="sorted", batch_size=bs, max_epoch=2,
                    use_amp=False, num_workers=0, best_model_criterion=[["valid", "loss", "min"]],
                    keep_nbest_models=1, use_preprocessor=False)
        tag = f"bs{bs}_eps{eps}"
        (tmp / f"{tag}.yaml").write_text(yaml.safe_dump(conf))
        def cmd(out, ngpu):
            return ["--config", str(tmp / f"{tag}.yaml"), "--output_dir", str(out), "--ngpu", str(ngpu),
                    "--token_list", str(tmp / "tokens.txt"), "--input_size", "80",
                    "--train_data_path_and_name_and_type", f"{tr}/feats.scp,speech,npy",
                    "--train_data_path_and_name_and_type", f"{tr}/text,text,text_int",
                    "--train_shape_file", f"{tr}/speech_shape",
                    "--valid_data_path_and_name_and_type", f"{dv}/feats.scp,speech,npy",
                    "--valid_data_path_and_name_and_type", f"{dv}/text,text,text_int",
                    "--valid_shape_file", f"{dv}/speech_shape"]
        ASRTask.main(cmd=cmd(tmp / f"one_{tag}", 1))
        ASRTask.main(cmd=cmd(tmp / f"two_{tag}", 2) + ["--dist_backend", "gloo", "--multiprocessing_distributed", "true"])
        c1 = torch.load(tmp / f"one_{tag}" / "checkpoint.pth", map_location="cpu", weights_only=True)
        c2 = torch.load(tmp / f"two_{tag}" / "checkpoint.pth", map_location="cpu", weights_only=True)
        for e in (1, 2):
            for ph in ("train", "valid"):
                a, b = c1["reporter"]["stats"][e][ph], c2["reporter"]["stats"][e][ph]
                print(tag, e, ph, {k: (round(a[k], 6), round(b[k], 6)) for k in ("loss", "loss_ctc", "loss_att") if k in a}, flush=True)
        worst = sorted(((float((c1["model"][k].float() - c2["model"][k].float()).abs().max()), k) for k in c1["model"]), reverse=True)[:4]
        print(tag, "param max abs diff", worst, flush=True)

if __name__ == "__main__":
    main()
