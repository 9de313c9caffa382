'use strict';
// cpu_bench.js -- the JS CPU integrator (rt0_cpu.js) on worker_threads.
// BASELINE / TEST INFRASTRUCTURE ONLY (see rt0_cpu.js).
//
// node cpu_bench.js <configs.json> <config> <W> <H> <threads> <mode> ...
//   mode "image" <frame0> <n> <out.f32>  : passes frame0..frame0+n-1 of the whole
//                                          image, RGBA f32 rows bottom-up -> file
//   mode "bench" <y0> <y1> <seconds>     : rows [y0,y1) split over the threads,
//                                          [--constants JSON] overrides constants,
//                                          successive passes until the deadline;
//                                          prints {"samples", "seconds", "msamples_s", ...}
const os = require('os');
const fs = require('fs');
const path = require('path');
const { Worker, isMainThread, parentPort, workerData } = require('worker_threads');
const { CpuRenderer } = require('./rt0_cpu.js');

function makeRenderer(d) {
  const cfgs = JSON.parse(fs.readFileSync(d.configs, 'utf8'));
  const cfg = cfgs.configs.find((c) => c.name === d.config);
  if (!cfg) throw new Error('no config ' + d.config);
  if (d.constants) cfg.constants = Object.assign({}, cfg.constants || {}, d.constants);
  return new CpuRenderer(cfg, cfgs.cornell_lines, cfgs.default_camera, d.W, d.H);
}

if (!isMainThread) {
  const d = workerData;
  const r = makeRenderer(d);
  if (d.mode === 'image') {
    const buf = r.render(d.frame0, d.n, d.y0, d.y1);
    parentPort.postMessage({ y0: d.y0, buf }, [buf.buffer]);
  } else {
    const t0 = Date.now();
    let samples = 0, frame = 1;
    while (Date.now() - t0 < d.seconds * 1000) {
      r.render(frame++, 1, d.y0, d.y1);
      samples += (d.y1 - d.y0) * d.W;
    }
    parentPort.postMessage({ samples, isect: r.nIsect });
  }
} else {
  const a = process.argv.slice(2);
  const base = { configs: path.resolve(a[0]), config: a[1], W: +a[2], H: +a[3] };
  const ci = a.indexOf('--constants');  // optional JSON of constant overrides (bench workloads)
  if (ci >= 0) base.constants = JSON.parse(a[ci + 1]);
  const threads = +a[4] || os.cpus().length;
  const mode = a[5];
  const split = (y0, y1) => {
    const out = [];
    const n = Math.max(1, Math.min(threads, y1 - y0));
    for (let i = 0; i < n; i++) {
      const lo = y0 + Math.floor(((y1 - y0) * i) / n), hi = y0 + Math.floor(((y1 - y0) * (i + 1)) / n);
      if (hi > lo) out.push([lo, hi]);
    }
    return out;
  };
  const run = (jobs) => Promise.all(jobs.map((wd) => new Promise((res, rej) => {
    const w = new Worker(__filename, { workerData: wd });
    w.on('message', res);
    w.on('error', rej);
  })));
  if (mode === 'image') {
    const frame0 = +a[6], n = +a[7], out = a[8];
    run(split(0, base.H).map(([y0, y1]) => Object.assign({ mode, frame0, n, y0, y1 }, base))).then((parts) => {
      const img = new Float32Array(base.W * base.H * 4);
      for (const p of parts) img.set(p.buf, p.y0 * base.W * 4);
      fs.writeFileSync(out, Buffer.from(img.buffer));
      console.log(JSON.stringify({ ok: true, threads }));
    }).catch((e) => { console.error(e); process.exit(1); });
  } else {
    const y0 = +a[6], y1 = +a[7], seconds = +a[8];
    const t0 = process.hrtime.bigint();
    run(split(y0, y1).map(([lo, hi]) => Object.assign({ mode, y0: lo, y1: hi, seconds }, base))).then((parts) => {
      const dt = Number(process.hrtime.bigint() - t0) / 1e9;
      const samples = parts.reduce((s, p) => s + p.samples, 0);
      console.log(JSON.stringify({
        samples, seconds: dt, msamples_s: samples / dt / 1e6, threads: parts.length,
        cpu: os.cpus()[0].model, node: process.version,
      }));
    }).catch((e) => { console.error(e); process.exit(1); });
  }
}
