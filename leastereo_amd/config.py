"""Model arguments, field-compatible with config_utils/leastereo_args.py:4-40 and
config_utils/predict_args.py:4-28 (same names, defaults and argparse flags)."""
from __future__ import annotations

import argparse
import os
from dataclasses import dataclass

ARCH_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "architecture")


@dataclass
class LEAStereoArgsNoArch:
    fea_num_layers: int = 6
    mat_num_layers: int = 12
    fea_filter_multiplier: int = 8
    mat_filter_multiplier: int = 8
    fea_block_multiplier: int = 4
    mat_block_multiplier: int = 4
    fea_step: int = 3
    mat_step: int = 3


@dataclass
class LEAStereoArgs(LEAStereoArgsNoArch):
    net_arch_fea: str = None
    cell_arch_fea: str = None
    net_arch_mat: str = None
    cell_arch_mat: str = None
    maxdisp: int = 192
    cuda: bool = True


def default_arch_args(args: LEAStereoArgs) -> LEAStereoArgs:
    """Fill unset .npy paths with the SceneFlow search result shipped in data/
    (run/sceneflow/best/architecture/*.npy of the reference)."""
    for field, fname in (("net_arch_fea", "feature_network_path.npy"),
                         ("cell_arch_fea", "feature_genotype.npy"),
                         ("net_arch_mat", "matching_network_path.npy"),
                         ("cell_arch_mat", "matching_genotype.npy")):
        if getattr(args, field) is None:
            setattr(args, field, os.path.join(ARCH_DIR, fname))
    return args


def add_leastereo_args_without_arch(parser: argparse.ArgumentParser):
    for name, default in LEAStereoArgsNoArch().__dict__.items():
        parser.add_argument("--" + name, type=int, default=default)


def add_leastereo_args(parser: argparse.ArgumentParser):
    add_leastereo_args_without_arch(parser)
    for name in ("net_arch_fea", "cell_arch_fea", "net_arch_mat", "cell_arch_mat"):
        parser.add_argument("--" + name, default=None, type=str)


def obtain_predict_args(argv=None):
    """predict_args.py:4-28: same flags.  (--cuda keeps the reference's
    ``type=bool`` quirk: any non-empty string enables it.)"""
    parser = argparse.ArgumentParser(description="LEStereo Prediction (MI355X)")
    parser.add_argument("--crop_height", type=int, required=True, help="crop height")
    parser.add_argument("--crop_width", type=int, required=True, help="crop width")
    parser.add_argument("--maxdisp", type=int, default=192, help="max disp")
    parser.add_argument("--resume", type=str, default="", help="resume from saved model")
    parser.add_argument("--cuda", type=bool, default=False, help="use cuda?")
    parser.add_argument("--data_path", type=str, required=True, help="data root")
    parser.add_argument("--test_list", type=str, required=True, help="training list")
    parser.add_argument("--save_path", type=str, default="./result/", help="location to save result")
    for flag in ("sceneflow", "kitti2012", "kitti2015", "middlebury", "satellite", "mvs3d",
                 "new_tagil", "whu"):
        parser.add_argument("--" + flag, type=int, default=0)
    parser.add_argument("--precision", choices=("f32", "bf16"), default="f32",
                        help="matching-net arithmetic (bf16: configs 3/4; not in the reference)")
    add_leastereo_args(parser)
    return parser.parse_args(argv)
