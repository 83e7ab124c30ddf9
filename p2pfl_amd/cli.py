"""Command-line interface: ``python -m p2pfl_amd <command>`` (or the ``p2pfl-amd`` script).

Reference: p2pfl/cli.py -- the ``experiment list`` / ``experiment run``
commands with unknown arguments passed through to the example, and the
``login`` / ``remote`` / ``launch`` placeholders.  Adds ``info`` (device,
native extension and kernel availability).
"""

from __future__ import annotations

import ast
import importlib
import os
import subprocess
import sys
from typing import Dict, List

import typer
from rich.console import Console
from rich.table import Table

app = typer.Typer(help="p2pfl_amd: decentralized federated learning on AMD Instinct MI355X.", no_args_is_help=True)
exp_app = typer.Typer(help="Run the bundled experiments.", no_args_is_help=True)
app.add_typer(exp_app, name="experiment")
console = Console()

EXAMPLES_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "examples")


def available_examples() -> Dict[str, str]:
    """name -> first line of the module docstring (parsed, never imported)."""
    out: Dict[str, str] = {}
    for fn in sorted(os.listdir(EXAMPLES_DIR)):
        if not fn.endswith(".py") or fn.startswith("_"):
            continue
        with open(os.path.join(EXAMPLES_DIR, fn), encoding="utf-8") as f:
            doc = ast.get_docstring(ast.parse(f.read())) or ""
        out[fn[:-3]] = doc.strip().splitlines()[0] if doc.strip() else ""
    return out


@exp_app.command("list")
def list_examples() -> None:
    """List the available examples."""
    table = Table(title="Available examples")
    table.add_column("Experiment", style="cyan", no_wrap=True)
    table.add_column("Description")
    for name, desc in available_examples().items():
        table.add_row(name, desc)
    console.print(table)


@exp_app.command("run", context_settings={"allow_extra_args": True, "ignore_unknown_options": True})
def run(ctx: typer.Context, example: str = typer.Argument(..., help="example name (see `experiment list`)")) -> None:
    """Run an example; extra arguments are passed through to it."""
    if example not in available_examples():
        console.print(f"[bold red]Unknown example {example!r}.[/bold red] Use [green]experiment list[/green].")
        raise typer.Exit(code=1)
    cmd: List[str] = [sys.executable, "-m", f"p2pfl_amd.examples.{example}", *ctx.args]
    console.print(f"[bold yellow]Running example {example}...[/bold yellow]")
    # a child process (never exec): the CLI itself has not touched the GPU
    rc = subprocess.call(cmd)
    if rc == 0:
        console.print(f"[bold green]Example {example} completed.[/bold green]")
    else:
        console.print(f"[bold red]Example {example} failed (exit {rc}).[/bold red]")
    raise typer.Exit(code=rc)


@app.command()
def info() -> None:
    """Show devices, the native extension and its kernels."""
    import torch

    from p2pfl_amd import ops

    table = Table(title="p2pfl_amd")
    table.add_column("item", style="cyan")
    table.add_column("value")
    table.add_row("torch", torch.__version__)
    table.add_row("hip", str(getattr(torch.version, "hip", None)))
    n = torch.cuda.device_count()
    table.add_row("devices", str(n))
    for i in range(n):
        table.add_row(f"  cuda:{i}", torch.cuda.get_device_name(i))
    table.add_row("native extension", "loaded" if ops.available() else "missing (run `python setup.py build_ext --inplace`)")
    if ops.available():
        ext = ops.ext()
        kernels = sorted(k for k in dir(ext) if not k.startswith("_"))
        kernels += sorted(f"cnn.{k}" for k in dir(ext.cnn) if not k.startswith("_"))
        table.add_row("kernels", ", ".join(kernels))
    console.print(table)


def _not_yet(what: str) -> None:
    console.print(f"[bold yellow]{what}: not implemented (the reference ships this as a placeholder too).[/bold yellow]")


@app.command()
def login(token: str = typer.Option("", help="API token")) -> None:
    """Authenticate against a p2pfl platform (placeholder)."""
    _not_yet("login")


@app.command()
def remote() -> None:
    """Interact with a remote node (placeholder)."""
    _not_yet("remote")


@app.command()
def launch() -> None:
    """Launch a new node (placeholder)."""
    _not_yet("launch")


def main() -> None:
    app()


if __name__ == "__main__":
    main()
