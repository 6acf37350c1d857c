"use strict";
/**
 * Per-call cost of three ways to hand out one promise per verifySignatureSets call, in a
 * pipeline like the Node drop-in's: packages of 32,768 calls, each package settled DEPTH
 * packages after it was issued, every call awaited by a caller `.then` (node 12).
 *   mode 0  page promise + `.then(pick[i])` per call (rounds 3-5)
 *   mode 1  `new Promise(exec)` per call, resolve and reject kept
 *   mode 2  `new Promise(exec)` per call, resolve kept (round 6)
 * Run: node tools/node_promise_floor.js <mode> [depth]
 */
const PKG = 32768, DEPTH = +(process.argv[3] || 5), NPKG = 60, PAGE = 8192;
const mode = +process.argv[2];
let RES, REJ; function EXEC(r, j) { RES = r; REJ = j; }
const PICK = []; for (let i = 0; i < PAGE; i++) PICK.push((pg) => { const s = pg.st[i]; if (s === 2) throw Error("x"); return s === 1; });
const sets = []; for (let i = 0; i < 1024; i++) sets.push({type: "single", pubkey: new Uint8Array(96), signingRoot: new Uint8Array(32), signature: new Uint8Array(96)});
let done = 0;
const onV = (ok) => { done++; };
function issue() {
  const pages = [];
  let pg = null;
  for (let i = 0; i < PKG; i++) {
    if (pg === null || pg.n === PAGE) {
      pg = {n: 0, st: null, sets: [], res: [], rej: [], p: null, r: null};
      if (mode === 0) pg.p = new Promise((r) => { pg.r = r; });
      pages.push(pg);
    }
    const s = [sets[i & 1023]]; const o = {batchable: true};
    let p;
    pg.sets.push(s);
    if (mode === 0) p = pg.p.then(PICK[pg.n]);
    else { p = new Promise(EXEC); pg.res.push(RES); if (mode === 1) pg.rej.push(REJ); }
    pg.n++;
    p.then(onV, null);
  }
  return pages;
}
function settle(pages) {
  for (const pg of pages) {
    if (mode === 0) { pg.st = new Int8Array(pg.n).fill(1); pg.r(pg); }
    else { const res = pg.res; for (let k = 0; k < pg.n; k++) { const f = res[k]; res[k] = undefined; if (mode === 1) pg.rej[k] = undefined; f(true); } }
  }
}
(async () => {
  const q = [];
  let t0 = 0;
  for (let k = 0; k < NPKG; k++) {
    if (k === 10) t0 = process.hrtime.bigint();
    q.push(issue());
    if (q.length > DEPTH) settle(q.shift());
    await new Promise((r) => setImmediate(r));
  }
  const us = Number(process.hrtime.bigint() - t0) / 1e3 / ((NPKG - 10) * PKG);
  console.log("mode", mode, "depth", DEPTH, "us/call", us.toFixed(3));
})();
