#!/usr/bin/env python
"""Train DCUE on MI355X through the reference's trainer API (dcrecommend.nn.dcue.DCUE).

The reference's README describes train_*.py drivers that build the datasets and call the trainer;
this is that driver for the MI355X build:

  python train_dcue.py --triplets triplets.csv --metadata metadata.csv --save-dir models/
  python train_dcue.py --synthetic --num-epochs 1 --save-dir /tmp/dcue   # self-contained demo

triplets: (user_id, song_id, score) by column position (datasets/dcuedataset.py:229,238);
metadata: song_id in column 1 and a `data_mel` column of torch.save'd [128, T] tensors
(datasets/dcueitemset.py:46,50). Arguments mirror DCUE's constructor (nn/dcue.py:47-50).
"""
import argparse
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "amplifai-deepcontentrecommenders_amd"))

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
import torch  # noqa: E402


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--triplets")
    ap.add_argument("--metadata")
    ap.add_argument("--save-dir", default="models")
    ap.add_argument("--synthetic", action="store_true",
                    help="generate a small synthetic interaction set and spectrogram files")
    ap.add_argument("--synthetic-users", type=int, default=60)
    ap.add_argument("--synthetic-tracks", type=int, default=120)
    ap.add_argument("--synthetic-pairs", type=int, default=1500)
    ap.add_argument("--feature-dim", type=int, default=100)  # DCUE's default, nn/dcue.py:44
    ap.add_argument("--conv-hidden", type=int, default=128)
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--neg-batch-size", type=int, default=20)
    ap.add_argument("--u-embdim", type=int, default=300)
    ap.add_argument("--margin", type=float, default=0.2)
    ap.add_argument("--lr", type=float, default=1e-5)
    ap.add_argument("--optimize", choices=["adam", "sgd", "ranger"], default="adam",
                    help="DCUE(optimize=...): nn/dcue.py:143-157")
    ap.add_argument("--model-type", default="truedcuemel1dbn", help="DCUE(model_type=...): dcue/dcue.py:49-59")
    ap.add_argument("--weight-decay", type=float, default=0.0)
    ap.add_argument("--num-epochs", type=int, default=90)
    ap.add_argument("--eval-pct", type=float, default=0.025)
    ap.add_argument("--val-pct", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=0)
    return ap.parse_args(argv)


def synthetic_data(n_users, n_tracks, n_pairs, out_dir, seed):
    """Unique (user, song) pairs and fp16-representable 131-frame spectrograms on disk."""
    rs = np.random.RandomState(seed)
    pairs = set()
    while len(pairs) < n_pairs:
        pairs.add((int(rs.randint(n_users)), int(rs.randint(n_tracks))))
    pairs = sorted(pairs)
    trip = pd.DataFrame({"user_id": ["u%06d" % u for u, _ in pairs],
                         "song_id": ["S%07d" % s for _, s in pairs],
                         "score": rs.randint(1, 10, size=len(pairs))})
    songs = sorted(set(trip["song_id"]))
    gen = torch.Generator().manual_seed(seed)
    paths = []
    for k, _ in enumerate(songs):
        p = os.path.join(out_dir, "mel_%06d.pt" % k)
        torch.save(torch.randn(128, 131, generator=gen).half().float(), p)
        paths.append(p)
    meta = pd.DataFrame({"idx": np.arange(len(songs)), "song_id": songs, "data_mel": paths})
    return trip, meta


def main(argv=None):
    args = parse(argv)
    from dcrecommend.datasets.dcuedataset import DCUEDataset
    from dcrecommend.datasets.dcueitemset import DCUEItemset
    from dcrecommend.datasets.dcuepredset import DCUEPredset
    from dcrecommend.nn.dcue import DCUE

    np.random.seed(args.seed)
    torch.manual_seed(args.seed)
    if args.synthetic:
        mel_dir = tempfile.mkdtemp(prefix="dcue_mel_")
        trip, meta = synthetic_data(args.synthetic_users, args.synthetic_tracks, args.synthetic_pairs,
                                    mel_dir, args.seed)
        triplets_path, metadata_path = "<synthetic>", mel_dir
    else:
        if not args.triplets or not args.metadata:
            raise SystemExit("--triplets and --metadata are required (or --synthetic)")
        trip = pd.read_csv(args.triplets)
        meta = pd.read_csv(args.metadata)
        triplets_path, metadata_path = args.triplets, args.metadata

    train = DCUEDataset(trip.copy(), meta, neg_samples=args.neg_batch_size, split="train")
    val = DCUEDataset(trip.copy(), meta, neg_samples=args.neg_batch_size, split="val")
    test = DCUEDataset(trip.copy(), meta, neg_samples=args.neg_batch_size, split="test")
    pred = DCUEPredset(trip.copy(), meta, split="val")
    truth = DCUEPredset(trip.copy(), meta, split="train")
    items = DCUEItemset(trip.copy(), meta)
    dcue = DCUE(feature_dim=args.feature_dim, conv_hidden=args.conv_hidden, batch_size=args.batch_size,
                neg_batch_size=args.neg_batch_size, u_embdim=args.u_embdim, margin=args.margin, lr=args.lr,
                weight_decay=args.weight_decay, num_epochs=args.num_epochs, eval_pct=args.eval_pct,
                val_pct=args.val_pct, optimize=args.optimize, model_type=args.model_type)
    dcue.fit(train, val, test, pred, truth, items, len(train.user_index), len(train.item_index),
             triplets_path, metadata_path, args.save_dir)
    return dcue


if __name__ == "__main__":
    main()
