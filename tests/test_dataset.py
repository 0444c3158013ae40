"""Host-side input pipeline (CPU): sample construction and padding of the reference's dataset schema
(src/custom_dataset.py:9-132), restated in ergm_amd.dataset."""
import torch

from ergm_amd.dataset import DialogueDataset, PadCollate

SP1, SP2, EOS = 98, 99, 97


def _schema():
    # two dialogues; dialogue 0 has two utterances, dialogue 1 one (too long -> skipped) + one short
    txt = [
        [[[1, 2, 3], [4, 5]], [[6, 7], [8], [9, 10, 11]]],
        [[list(range(20))] * 60, [[12, 13]]],
    ]
    label = [
        [[50, 51, 30, 31, 60, 61], [50, 51, 40, 41, 42, 43, 44, 45, 46, 47, 60, 61]],
        [[50, 51, 1, 60, 61], [50, 51, 2, 60, 61]],
    ]
    img = [[torch.full((8,), 0.5)], [torch.full((8,), -1.0)]]
    aud = [[torch.full((8,), 2.0)], [torch.full((8,), 3.0)]]
    context = [[[70, 71], [72]], [[73], [74, 75, 76]]]
    emo = [[3, 4], [5, 6]]
    return {"txt": txt, "img": img, "aud": aud, "label": label}, {"context": context, "label": emo}


def test_sample_construction_follows_reference_rules():
    data, ctx = _schema()
    ds = DialogueDataset(data, ctx, sp1_id=SP1, sp2_id=SP2, eos_id=EOS)
    assert len(ds) == 3  # the 1200-token utterance is dropped (>= 1024, src/custom_dataset.py:50-51)
    ids, tt, lm, vis, aud, c, e = ds[0]
    assert ids == [1, 2, 3, 4, 5]
    assert tt == [SP1, SP1, SP1, SP2, SP2]
    assert lm == [-100, -100, 30, 31, EOS]          # target[2:-2] + eos, right-aligned
    assert torch.equal(vis, torch.full((8,), 0.5)) and torch.equal(aud, torch.full((8,), 2.0))
    assert c == [70, 71] and e == 3
    ids, tt, lm, *_ = ds[1]                          # target longer than the input: input eos-padded
    assert lm == [40, 41, 42, 43, 44, 45, 46, 47, EOS]
    assert ids == [6, 7, 8, 9, 10, 11, EOS, EOS, EOS]
    assert tt == [SP1, SP1, SP2, SP1, SP1, SP1, SP1, SP1, SP1]
    assert ds[2][6] == 6


def test_pad_collate():
    data, ctx = _schema()
    ds = DialogueDataset(data, ctx, sp1_id=SP1, sp2_id=SP2, eos_id=EOS)
    b = PadCollate(eos_id=EOS, pad_multiple=4)([ds[0], ds[1], ds[2]])
    assert b["input_ids"].shape == (3, 12)           # longest 9, rounded up to a multiple of 4
    assert b["input_ids"][0, 5:].eq(EOS).all() and b["token_type_ids"][0, 5:].eq(EOS).all()
    assert b["labels"][0, 5:].eq(-100).all() and b["labels"][1, 8] == EOS
    assert b["caption_ids"][2, :3].tolist() == [74, 75, 76] and b["caption_ids"][2, 3:].eq(EOS).all()
    assert b["visual_feat"].shape == (3, 8) and b["audio_feat"][2, 0] == 3.0
    assert b["emotion_labels"].tolist() == [3, 4, 6]


def _ref_fixture():
    import json
    import os
    import numpy as np
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dataset_ref.npz"))
    return {k: z[k] for k in z.files}, json


def test_matches_reference_dataset_and_collate_outputs():
    """DialogueDataset / PadCollate against the reference's own CustomDataset + PadCollate outputs
    (tests/golden/dataset_ref.npz, written by tests/golden/make_golden.py from src/custom_dataset.py on
    synthetic pickles; one dialogue per file because of the reference's [:1] debug slices)."""
    rec, json = _ref_fixture()
    eos, sp1, sp2 = int(rec["eos"]), int(rec["sp1"]), int(rec["sp2"])
    data = {"txt": [], "img": [], "aud": [], "label": []}
    cl = {"context": [], "label": []}
    i = 0
    while f"dlg{i}_json" in rec:
        d = json.loads(bytes(rec[f"dlg{i}_json"]).decode())
        for k in data:
            data[k] += d["data"][k]
        for k in cl:
            cl[k] += d["cl"][k]
        i += 1
    ds = DialogueDataset(data, cl, sp1_id=sp1, sp2_id=sp2, eos_id=eos)
    n = int(rec["n"])
    assert len(ds) == n
    for r in range(n):
        ids, tt, lm, vis, aud, ctx, emo = ds[r]
        L = int(rec["lengths"][r])
        assert ids == rec["sample_input_ids"][r, :L].tolist()
        assert tt == rec["sample_token_type_ids"][r, :L].tolist()
        assert lm == rec["sample_labels"][r, :L].tolist()
        assert torch.equal(vis, torch.from_numpy(rec["img0"][r])) and torch.equal(aud, torch.from_numpy(rec["aud0"][r]))
        c = rec["sample_context"][r]
        assert ctx == c[c != -7].tolist() and emo == int(rec["emotion"][r])
    # the reference model reads imgs[i][0] of the per-token copies: the dialogue's first visual row
    assert (rec["n_img_rows"] == rec["lengths"]).all()
    coll = PadCollate(eos_id=eos)
    for bi, rows in ((0, list(range(n))), (1, [1, 2])):
        b = coll([ds[r] for r in rows])
        for key in ("input_ids", "token_type_ids", "labels"):
            assert b[key].tolist() == rec[f"batch{bi}_{key}"].tolist(), (bi, key)


def test_product_schedule_matches_transformers():
    """ergm_amd.optim's poly-decay schedule (src/main.py:93-95, power 2) against the LRs transformers'
    get_polynomial_decay_schedule_with_warmup produced (tests/golden/adamw_sched.npz)."""
    import os
    import numpy as np
    from ergm_amd.optim import polynomial_decay_lr_lambda
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "adamw_sched.npz"))
    lr, warm, total = z["sched_args"]
    f = polynomial_decay_lr_lambda(int(warm), int(total), float(lr), power=2.0)
    got = [float(lr) * f(k) for k in range(len(z["sched_lrs"]))]
    assert np.allclose(got, z["sched_lrs"], rtol=1e-12, atol=0)
    f1 = polynomial_decay_lr_lambda(1, 5, 2e-5, power=2.0)
    assert np.allclose([2e-5 * f1(k) for k in range(3)], z["lrs"], rtol=1e-12, atol=0)
