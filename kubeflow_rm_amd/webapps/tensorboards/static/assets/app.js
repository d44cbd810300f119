// TensorBoards web app frontend (reference crud-web-apps/tensorboards/frontend): table (common
// resource table, polled), create from a PVC path (pvc://<claim>/<path>) or an object-store URL
// (s3:// gs://), PodDefault configurations, delete, connect at /tensorboard/<ns>/<name>/.
// `TWA` holds the pure parts (columns, logspath building, validation) for the node tests.
(function (global) {
  "use strict";
  const kf = global.kf || (typeof require !== "undefined" ? require("../../../crud_backend/static/kf.js") : null);

  const TWA = {
    // confirm dialog (pages/index/index.component.ts)
    dialogs: {
      delete: (name) => ({ title: `Are you sure you want to delete this Tensorboard : ${name} ?`, message: "",
                           accept: "DELETE", confirmColor: "warn", cancel: "CANCEL", error: "", applying: "DELETING",
                           width: "600px" }),
    },
    columns(allNamespaces) {
      const cols = [
        { title: "Status", value: (r) => r.status.phase, html: (r) => kf.statusIcon(r.status) },
        { title: "Name", value: (r) => r.name },
      ];
      if (allNamespaces) cols.push({ title: "Namespace", value: (r) => r.namespace });
      cols.push({ title: "Logspath", value: (r) => r.logspath }, { title: "Created at", kind: "date", value: (r) => r.age });
      return cols;
    },
    logspath(kind, pvc, path) {
      const p = String(path || "").trim();
      return kind === "pvc" ? `pvc://${pvc}/${p.replace(/^\/+/, "")}` : p;
    },
    // pages/index/index.component.ts processIncomingData: per-row action states (delete is held while
    // the object terminates, connect only once the server is ready) and the age cell's tooltip.
    process(rows) {
      return rows.map((t) => {
        const r = JSON.parse(JSON.stringify(t));
        r.deleteAction = r.status.phase === "terminating" ? "terminating" : "ready";
        r.connectAction = r.status.phase === "ready" ? "ready" : "unavailable";
        if (r.age && typeof r.age === "object") { r.ageValue = r.age.uptime; r.ageTooltip = r.age.timestamp; }
        return r;
      });
    },
    // Optimistic row state after an accepted DELETE, until the next poll sees the object go.
    markDeleting(r) {
      r.status = Object.assign({}, r.status, { phase: "terminating", message: "Preparing to delete the Tensorboard object..." });
      r.deleteAction = "unavailable";
      return r;
    },
    // pages/form/form.component.ts: names already taken in the namespace are rejected client-side.
    validate(name, kind, pvc, path, taken) {
      const errs = [];
      const n = kf.validators.name(name);
      if (n) errs.push(n);
      else if (taken && taken.has(name)) errs.push(`TensorBoard ${name} already exists`);
      if (kind === "pvc" && !pvc) errs.push("Select a PVC");
      if (kind !== "pvc" && !/^(s3|gs):\/\/[^/]+/.test(String(path || "").trim())) errs.push("Object store paths look like s3://bucket/path or gs://bucket/path");
      return errs;
    },
  };

  function app() {
    const $ = (id) => document.getElementById(id);
    let poller = null, table = null, rows = [];
    // "All namespaces" (index.component.ts polls getTensorBoards(ns) with an array): rows of every
    // namespace, merged, with a Namespace column; creating still targets one namespace.
    const ALL = "__all__";
    let list = [], allNs = false;
    async function namespaces() {
      try { list = (await kf.call("GET", "/api/namespaces")).namespaces; } catch (e) { list = kf.namespace() ? [kf.namespace()] : []; }
      $("ns").innerHTML = list.map((n) => `<option value="${kf.esc(n)}">${kf.esc(n)}</option>`).join("") +
        (list.length > 1 ? `<option value="${ALL}">All namespaces</option>` : "");
      if (!kf.namespace() && list.length) kf.setNamespace(list[0]);
      $("ns").value = kf.namespace();
      $("ns").onchange = () => {
        allNs = $("ns").value === ALL;
        table = new kf.ResourceTable($("rows"), tableConfig());
        $("new").disabled = allNs;
        if (allNs) poller.reset(); else kf.setNamespace($("ns").value);
      };
    }
    function tableConfig() {
      return {
        columns: TWA.columns(allNs), empty: allNs ? "No TensorBoards in any namespace." : "No TensorBoards in this namespace.",
        actions: [{ name: "connect", label: "Connect", enabled: (r) => r.connectAction === "ready" },
                  { name: "delete", label: "Delete", enabled: (r) => r.deleteAction === "ready" }],
        onAction: async (name, r) => {
          if (name === "connect") window.open(`/tensorboard/${r.namespace}/${r.name}/`);
          if (name === "delete") {
            const ok = await kf.confirmDialog(TWA.dialogs.delete(r.name), () => kf.call("DELETE", `/api/namespaces/${r.namespace}/tensorboards/${r.name}`));
            if (ok === "accept") { TWA.markDeleting(r); table.setRows(rows); }
            poller.reset();
          }
        },
      };
    }
    async function refresh() {
      const nss = allNs ? list : [kf.namespace()].filter(Boolean);
      if (!nss.length) return null;
      const per = await Promise.all(nss.map(async (ns) =>
        (await kf.call("GET", `/api/namespaces/${ns}/tensorboards`)).tensorboards.map((t) => Object.assign({ namespace: ns }, t))));
      rows = TWA.process([].concat(...per));
      table.setRows(rows);
      return rows.map((t) => [t.namespace, t.name, t.status.phase]);
    }
    async function open() {
      const ns = kf.namespace();
      const [{ pvcs }, { poddefaults }] = await Promise.all([kf.call("GET", `/api/namespaces/${ns}/pvcs`),
        kf.call("GET", `/api/namespaces/${ns}/poddefaults`)]);
      $("f-pvc").innerHTML = pvcs.map((p) => `<option>${kf.esc(p)}</option>`).join("");
      $("f-configs").innerHTML = poddefaults.map((pd) => `<label class="muted"><input type="checkbox" value="${kf.esc(pd.label)}"> ${kf.esc(pd.desc)}</label><br>`).join("");
      // form.component.ts: object store is the default; the PVC picker shows only for PVC storage
      const kind = () => { $("f-pvc-row").hidden = $("f-kind").value !== "pvc"; };
      $("f-kind").onchange = kind; kind();
      $("f-error").textContent = "";
      $("dlg").showModal();
    }
    async function submit(ev) {
      if (ev.submitter && ev.submitter.value !== "ok") return;
      ev.preventDefault();
      const ns = kf.namespace(), kind = $("f-kind").value;
      const taken = new Set(rows.filter((r) => r.namespace === ns).map((r) => r.name));
      const errs = TWA.validate($("f-name").value, kind, $("f-pvc").value, $("f-path").value, taken);
      if (errs.length) { $("f-error").textContent = errs.join("; "); return; }
      const logspath = TWA.logspath(kind, $("f-pvc").value, $("f-path").value);
      const configurations = [...$("f-configs").querySelectorAll("input:checked")].map((i) => i.value);
      try {
        await kf.call("POST", `/api/namespaces/${ns}/tensorboards`, { name: $("f-name").value, logspath, configurations });
        $("dlg").close(); kf.snack(`TensorBoard ${$("f-name").value} created`, "SUCCESS"); poller.reset();
      } catch (e) { $("f-error").textContent = e.message; }
    }
    (async function main() {
      poller = new kf.Poller(refresh);
      table = new kf.ResourceTable($("rows"), tableConfig());
      $("filter").oninput = (ev) => table.setFilter(ev.target.value);
      await namespaces();
      $("new").onclick = open;
      $("form").addEventListener("submit", submit);
      kf.onNamespace((ns) => { if (!allNs) { $("ns").value = ns; poller.reset(); } });
      poller.start();
    })();
  }

  global.TWA = TWA;
  if (typeof module !== "undefined" && module.exports) module.exports = TWA;
  else if (typeof document !== "undefined") app();
})(typeof window !== "undefined" ? window : globalThis);
