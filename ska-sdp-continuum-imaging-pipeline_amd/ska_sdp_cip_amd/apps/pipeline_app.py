"""
The pipeline app with the reference's command line (reference
src/ska_sdp_cip/apps/pipeline_app.py:17-116): measurement set in, dirty image
out as .npy; serial `invert_measurement_set` without a scheduler, else
`dask_invert_measurement_set` over the given client with the task list saved
as `task-list.json` (TaskMetrics). Flags are the reference's; what differs:

* `--dask-scheduler local` runs the distributed form on this node's GPUs
  through `dispatch.LocalGPUClient` (one worker per GPU); any other address
  needs dask.distributed (not installed in this image) and is passed to its
  `Client`, whose GPU workers must carry a `{"gpu": 1}` resource;
* the measurement set may be an .npz column file
  (`InMemoryMeasurementSet.save_npz`), since python-casacore is absent;
* `--stokes-on-device` forms Stokes I inside the gridder (raw columns to the
  GPU), serial or per distributed task.
"""

from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np

from .. import __version__
from ..invert import dask_invert_measurement_set, invert_measurement_set
from ..measurement_set import open_measurement_set
from ..task_metrics import TaskMetrics


def get_parser() -> argparse.ArgumentParser:
    """The CLI parser (reference :17-78, same arguments and defaults)."""
    parser = argparse.ArgumentParser(
        description="Launch the SKA continuum imaging pipeline",
        formatter_class=argparse.ArgumentDefaultsHelpFormatter,
    )
    parser.add_argument("--version", action="version", version=__version__)
    parser.add_argument("measurement_set", type=Path, help="Path to MeasurementSet v2 (or an .npz column file)")
    parser.add_argument("output_image", type=Path,
                        help="Path to output image, which is saved as a numpy array")
    imaging = parser.add_argument_group("imaging")
    imaging.add_argument("-n", "--num-pixels", type=int, required=True, help="Number of pixels across the image")
    imaging.add_argument("-p", "--pixel-size", type=float, required=True,
                         help="Pixel size in arcseconds at the image centre")
    imaging.add_argument("--stokes-on-device", action="store_true",
                         help="Form Stokes I inside the GPU gridder from the raw columns")
    dask = parser.add_argument_group("dask distribution")
    dask.add_argument("-d", "--dask-scheduler", type=str, default=None,
                      help="Optional address of a dask scheduler to use for distribution "
                           "('local': this node's GPUs, one worker each)")
    dask.add_argument("-rc", "--row-chunks", type=int, default=1, help="Number of row chunks to use for distribution")
    dask.add_argument("-fc", "--freq-chunks", type=int, default=None,
                      help="Number of frequency chunks to use for distribution. "
                           "If None, set this to the number of dask workers.")
    return parser


def _client(address: str):
    if address == "local":
        from ..dispatch import LocalGPUClient  # pylint: disable=import-outside-toplevel

        return LocalGPUClient()
    from dask.distributed import Client  # pylint: disable=import-outside-toplevel

    return Client(address)


def run_program(cli_args: list) -> None:
    """Run the app (reference :81-109); the function the tests call."""
    args = get_parser().parse_args(cli_args)
    mset = open_measurement_set(args.measurement_set)
    if args.dask_scheduler is None:
        img = invert_measurement_set(mset, num_pixels=args.num_pixels, pixel_size_asec=args.pixel_size,
                                     stokes_on_device=args.stokes_on_device)
    else:
        client = _client(args.dask_scheduler)
        if args.dask_scheduler == "local":
            with client, client.get_task_stream() as stream:
                img = dask_invert_measurement_set(mset, client, num_pixels=args.num_pixels,
                                                  pixel_size_asec=args.pixel_size, row_chunks=args.row_chunks,
                                                  freq_chunks=args.freq_chunks,
                                                  stokes_on_device=args.stokes_on_device)
        else:
            from dask.distributed import get_task_stream, performance_report  # pylint: disable=import-outside-toplevel

            with get_task_stream(client) as stream, performance_report(filename="dask-report.html"):
                img = dask_invert_measurement_set(mset, client, num_pixels=args.num_pixels,
                                                  pixel_size_asec=args.pixel_size, row_chunks=args.row_chunks,
                                                  freq_chunks=args.freq_chunks,
                                                  stokes_on_device=args.stokes_on_device)
        TaskMetrics(stream.data).save_json("task-list.json", indent=4, sort_keys=True)
    np.save(args.output_image.with_suffix(".npy"), img)


def main() -> None:
    """Entry point (reference :112-116)."""
    run_program(sys.argv[1:])


if __name__ == "__main__":
    sys.exit(main())
